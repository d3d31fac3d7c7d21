// Strip-walking first pair: conv1_1 -> relu -> conv1_2 -> relu [-> pool1] [+ the head split's skip-half partials]
// (unet.py:170-172 at full resolution, and conv1_5's share of cat1's conv1_2 half, unet.py:203).
//
// The tile-per-block pair kernel (conv3x3_pair_persist) runs its phases in lock step: all 8 waves evaluate conv1_1 on
// the tile's halo patch (VALU-heavy, a third of the patch is halo), meet at a barrier, run conv1_2, meet again, stage
// and store.  The matrix pipe idles through the first and last phase (MFMA busy 0.29).  Here a 2-wave workgroup walks
// a 32-pixel-wide column strip down a segment of rows and keeps a 4-row ring of conv1_1 output rows in LDS:
//   * per output row r it evaluates ONE new conv1_1 row (r + 2; 34 pixels for 32 outputs: the horizontal halo only,
//     no vertical recompute inside a segment) and conv1_2 row r from ring rows r-1 .. r+1;
//   * wave w owns output channels 32w .. 32w+31 of both convs, and holds its conv1_2 filter (18 K-steps x 2
//     fragments = 144 VGPRs) and conv1_1 filter in registers for the whole segment, so the only LDS reads in the
//     conv1_2 loop are the pixel fragments (2 per 4 MFMAs);
//   * the input rows (f32 frame -> bf16 8-channel chunks) go through an 8-row LDS ring, loaded a row ahead;
//   * one 128-thread barrier per output row; with 4 workgroups per CU the waves of other strips fill each SIMD's
//     gaps, so no phase of one strip stalls the matrix pipe of the CU;
//   * the epilogue works from registers: bias/affine/act, 16-byte stores of whole channel chunks (chunk_pair),
//     the 2x2 SAME max-pool from the previous row's registers and a DPP column exchange, and the head split's
//     per-tap partials (2 MFMAs on the bf16 outputs, handed to wave 0 through LDS a row later).
// Every MFMA sequence (conv1_1: 3 K-steps of 4 taps x 8 channels; conv1_2: granule 0 taps 0..8, granule 1 taps
// 0..8; head: channels 0..31 then 32..63) is the one the tile kernels run, so outputs, pool and partials are
// bit-identical to conv3x3_pair_persist (tests/test_gpu_parity.py::test_pair_strip_*).
#include "conv_common.h"

namespace vm {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

struct StripCfg {
  // 30 output columns per strip: the conv1_1 row then spans exactly 32 columns (-1 .. 30) = two 16-pixel MFMA
  // fragments (a 32-column strip needs 34, i.e. a third fragment for 2 columns); conv1_2's last fragment computes 2
  // columns it does not store
  static constexpr int SW = 30;                  // output columns per strip
  static constexpr int RC = SW + 2;              // conv1_1 columns per ring row (strip columns -1 .. 30)
  static constexpr int RW = 32;                  // ring row stride in pixels: a multiple of 8 keeps swz2 row-independent
  static constexpr int RSLOT = 4;                // conv1_1 rows in the ring (r-1 .. r+1 read, r+2 written)
  static constexpr int PLANE = RSLOT * RW * 64;  // one 32-channel granule plane (64-byte pixel rows)
  static constexpr int IW = SW + 4, ISLOT = 8;   // input ring: strip columns -2 .. 31, 16 bytes per pixel
  static constexpr int I_OFF = 2 * PLANE;
  static constexpr int X_OFF = I_OFF + ISLOT * IW * 16;  // head B operands: [row parity][wave][fp][lane] uint4
  static constexpr int K_OFF = X_OFF + 2 * 2 * 2 * 64 * 16;  // mul[64], add[64], bias1[64]
  static constexpr int H_OFF = K_OFF + 3 * 64 * 4;       // head A fragments [kk][lane] uint4
  static constexpr int RSZ = 2048;                       // raw input window staging (<= 2 DMA instructions), 2 slots
  static constexpr int R_OFF = H_OFF + 2 * 64 * 16;
  static constexpr int LDS = R_OFF + 2 * RSZ;
};

// XIN: 0 = bf16 frame of 8-channel pixels, 2 = f32 frame with x_c <= 8 channels (cstride <= 8)
// ACT: the epilogue's activation as a compile-time constant (a runtime switch per element made hipcc emit a branch
// tree per value, and this kernel is issue-bound, not MFMA-bound)
// XC: the f32 frame's channel count when known at compile time (7: the video path's cmp / bg / trimap frame), 0 =
// a.x_c at run time (a per-channel branch with its own LDS-load wait)
template <int XIN, int ACT, int ABL = 0, int PIN = 1, int XC = 0>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2)))
void conv3x3_pair_strip(ConvArgs a, int seg, int nseg, int nstrip) {
  using C = StripCfg;
  using T = uint16_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, q = lane >> 4;
  const int H = a.H, W = a.W;
  const int strip = blockIdx.x % nstrip, rest = blockIdx.x / nstrip;
  const int sg = rest % nseg, n = rest / nseg;
  const int c0 = strip * C::SW, s0 = sg * seg, s1 = min(s0 + seg, H);

  // filters in registers: conv1_2 K-step s = granule s / 9, tap s % 9 (chunk-major packing), conv1_1 K-step j =
  // taps 4j .. 4j+3 x 8 channels (tap-major, K_pad 128); rows = this wave's 32 output channels
  const T* wg = reinterpret_cast<const T*>(a.w);
  const T* w1 = reinterpret_cast<const T*>(a.w1);
  uint4 w2[18][2], w1f[3][2];
#pragma unroll
  for (int s = 0; s < 18; ++s)
#pragma unroll
    for (int f = 0; f < 2; ++f)
      w2[s][f] = *reinterpret_cast<const uint4*>(wg + (long)(32 * wave + 16 * f + col) * a.K_pad + s * 32 + q * 8);
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int f = 0; f < 2; ++f)
      w1f[j][f] = *reinterpret_cast<const uint4*>(w1 + (32 * wave + 16 * f + col) * 128 + j * 32 + q * 8);
  float* rk = reinterpret_cast<float*>(smem + C::K_OFF);
  if (tid < 64) {
    const int co = min(tid, a.cout - 1);
    const float sc = a.scale ? a.scale[co] : 1.f;
    rk[tid] = sc;
    rk[64 + tid] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
    rk[128 + tid] = a.bias1 ? a.bias1[tid] : 0.f;
  } else if (a.hd) {
    // head split: A fragments of the skip half's head filter, rows = taps (9 of 16), k = 8q + j <-> conv1_2 channel
    // (2kk + j/4)*16 + 4q + j%4, the order in which the epilogue's lanes hold their bf16 outputs (B operand)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint32_t u[4];
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const int j0 = 2 * jp, j1 = 2 * jp + 1;
        const int ch0 = (2 * kk + j0 / 4) * 16 + 4 * q + j0 % 4, ch1 = (2 * kk + j1 / 4) * 16 + 4 * q + j1 % 4;
        const float h0 = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + ch0] : 0.f;
        const float h1 = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + ch1] : 0.f;
        u[jp] = bf16x2_bits(h0, h1);
      }
      *reinterpret_cast<uint4*>(smem + C::H_OFF + (kk * 64 + lane) * 16) = make_uint4(u[0], u[1], u[2], u[3]);
    }
  }

  // ---- input rows: the window of strip columns -2 .. 33 of one frame row is contiguous in HBM (NHWC), so wave 0
  // fetches it with one or two LDS-DMA instructions (no registers held across the MFMA phases) into a 2-slot raw
  // staging ring, and a row later lanes 0..35 convert it to bf16 8-channel chunks (zero outside the frame) in the
  // 8-row input ring.  The descriptor covers ONE image, and the fetched bytes [ws, ws + nd KB) are clamped inside it
  // (ws = the window's first byte, moved right at the image start and left at its end), so no 16-byte piece ever
  // straddles the image bounds: every needed byte is fetched, none outside the tensor.  Rows outside the frame fetch
  // nothing (out-of-range offsets read as zeros).
  const int es = XIN == 2 ? 4 : 2, cs = a.x_cstride;
  const int pxb = cs * es, imgb = H * W * pxb;  // host: imgb >= 2 KB and < 2 GB
  const char* ximg = reinterpret_cast<const char*>(a.x) + ((long)a.x_coff + (long)n * H * W * cs) * es;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(ximg), 0, (uint32_t)imgb, 0x00020000);
  const int nd = (C::IW * pxb + 1023) / 1024;  // DMA instructions per row (host: <= 2)
  const uint32_t raw0 = __builtin_amdgcn_readfirstlane(lds_addr(smem + C::R_OFF));
  auto wstart = [&](int ir) __attribute__((always_inline)) {  // first fetched byte of row ir's window
    return min(max((ir * W + c0 - 2) * pxb, 0), imgb - nd * 1024);
  };
  auto dma_row = [&](int ir, int slot) __attribute__((always_inline)) {  // wave 0
    const bool ok = (unsigned)ir < (unsigned)H;
    const int base = wstart(ir) + lane * 16;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(raw0 + slot * C::RSZ);
    glds16(xrs, dst, ok ? base : OOB_INL);
    if (nd > 1) glds16(xrs, dst + 1024, ok ? base + 1024 : OOB_INL);
  };
  auto convert_row = [&](int ir, int slot) __attribute__((always_inline)) {  // wave 0, lanes 0..35
    if (lane < C::IW) {
      const int xc = c0 - 2 + lane;
      const bool ok = (unsigned)ir < (unsigned)H && (unsigned)xc < (unsigned)W;
      const char* rp = smem + C::R_OFF + slot * C::RSZ + (ok ? (ir * W + xc) * pxb - wstart(ir) : 0);
      uint4 v;
      if constexpr (XIN == 2) {
        float xz[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          xz[c] = c < (XC ? XC : a.x_c) ? *reinterpret_cast<const float*>(rp + 4 * c) : 0.f;
        v = Chunk<T>::pack(xz);
      } else {
        v = *reinterpret_cast<const uint4*>(rp);
      }
      *reinterpret_cast<uint4*>(smem + C::I_OFF + ((ir & 7) * C::IW + lane) * 16) = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };

  // ---- conv1_1 row jr (+ bias + relu; zero outside the frame = conv1_2's SAME padding) -> this wave's plane, slot jr&3
  T* y1b = a.y1 ? reinterpret_cast<T*>(a.y1) + a.y1_coff + ((long)n * H) * W * (long)a.y1_cstride : nullptr;
  const __amdgpu_buffer_rsrc_t y1rs = __builtin_amdgcn_make_buffer_rsrc(y1b, 0, 0x7ffffff0, 0x00020000);
  auto conv1 = [&](int jr) __attribute__((always_inline)) {
    // lane-derived addresses are recomputed per call (an opaque copy of the lane id): hoisted out of the row loop they
    // would hold a dozen registers the filters need
    int l = lane;
    asm volatile("" : "+v"(l));
    const int cl = l & 15, ql = l >> 4;
    const int cq16 = (ql & 1) ? 2 + (ql >> 1) : ql >> 1;
    const bool rin = (unsigned)jr < (unsigned)H;
    char* dst = smem + wave * C::PLANE + (jr & 3) * (C::RW * 64) + swz2(cl, cq16);
    float b1[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float4 bb = *reinterpret_cast<const float4*>(rk + 128 + 32 * wave + 16 * f + 4 * ql);
      b1[f][0] = bb.x; b1[f][1] = bb.y; b1[f][2] = bb.z; b1[f][3] = bb.w;
    }
    // input-ring byte offset of K-step j's tap (4j + ql, taps 9..11 -> 8) for ring column cl: the three input-row
    // offsets are uniform (scalar), the lane picks one (j = 0: tap ql, j = 1: tap 4 + ql, j = 2: tap 8)
    int ro[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) ro[d] = C::I_OFF + ((jr - 1 + d) & 7) * (C::IW * 16);
    const bool q3 = ql == 3, q01 = ql < 2;
    const int ib[3] = {(q3 ? ro[1] : ro[0]) + (cl + (q3 ? 0 : ql)) * 16,
                       (q01 ? ro[1] : ro[2]) + (cl + (q01 ? 1 + ql : ql - 2)) * 16, ro[2] + (cl + 2) * 16};
    // branch-free (one basic block with conv1_2's loop, so the two can interleave): rows outside the frame read the
    // input ring's zero rows and are masked to zero like columns outside it
#pragma unroll
    for (int fr = 0; fr < C::RC / 16; ++fr) {
      const int rc = fr * 16 + cl;  // ring column: strip column rc - 1
      f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        // unconditional: taps 9..11 (K-step 2, q > 0) read tap 8's pixel, whose finite values meet zero weights
        // (the products are zeros, as with a zero operand)
        const uint4 bv = *reinterpret_cast<const uint4*>(smem + ib[j] + fr * 256);
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          if constexpr (ABL & 1) asm volatile("" ::"v"(bv.x), "v"(w1f[j][f].x));
          else mma16<T>(w1f[j][f], bv, acc1[f]);
        }
      }
      const int cc = c0 - 1 + rc;
      const bool inside = rin && (unsigned)cc < (unsigned)W;
      uint2 pk[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        float v[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[jj] = fmaxf(acc1[f][jj] + b1[f][jj], 0.f);
        // outside the frame: +0 (masked on the packed pairs, the bits a +0 float converts to)
        pk[f].x = inside ? bf16x2_bits(v[0], v[1]) : 0u;
        pk[f].y = inside ? bf16x2_bits(v[2], v[3]) : 0u;
      }
      // swz2(16 fr + cl, c) = 1024 fr + swz2(cl, c): ((16 fr + cl) >> 1) & 3 == (cl >> 1) & 3
      const uint4 ck = chunk_pair(pk[0], pk[1]);
      *reinterpret_cast<uint4*>(dst + fr * 1024) = ck;
      if (a.y1) {  // conv1_1 itself (the training towers' select convs read it): this segment's rows, own columns
        const int c = c0 + rc - 1;
        const bool ok = jr >= s0 && jr < s1 && rc >= 1 && rc <= C::SW && c < W;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, ck), y1rs,
                                               ok ? ((int)__umul24(jr * W + c, a.y1_cstride) + 32 * wave + 8 * cq16) * 2 : OOB_INL, 0, 0);
      }
    }
  };

  const int ycs2 = a.y_cstride * 2;
  T* yrow0 = reinterpret_cast<T*>(a.y) + a.y_coff + ((long)n * H) * W * (long)a.y_cstride;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yrow0, 0, 0x7ffffff0, 0x00020000);
  const int PH = (H + 1) >> 1, PWd = (W + 1) >> 1;
  T* prow0 = a.py ? reinterpret_cast<T*>(a.py) + a.py_coff + ((long)n * PH) * PWd * (long)a.py_cstride : nullptr;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(prow0, 0, 0x7ffffff0, 0x00020000);
  uint2 prev[2][2];  // the even row's bf16 outputs [fp][f] (pool partner)

  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.hd ? a.hd + (long)n * H * W * 12 : nullptr), 0, 0x7ffffff0, 0x00020000);
  auto head_finish = [&](int r) __attribute__((always_inline)) {  // wave 0: row r's partials (wave 1's half via LDS)
    const uint4 ha0 = *reinterpret_cast<const uint4*>(smem + C::H_OFF + lane * 16);
    const uint4 ha1 = *reinterpret_cast<const uint4*>(smem + C::H_OFF + (64 + lane) * 16);
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) {
      const uint4 hb0 = *reinterpret_cast<const uint4*>(smem + C::X_OFF + ((((r & 1) * 2 + 0) * 2 + fp) * 64 + lane) * 16);
      const uint4 hb1 = *reinterpret_cast<const uint4*>(smem + C::X_OFF + ((((r & 1) * 2 + 1) * 2 + fp) * 64 + lane) * 16);
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
      mma16<T>(ha0, hb0, d);
      mma16<T>(ha1, hb1, d);
      const int p = fp * 16 + col, c = c0 + p;
      // a buffer store per fragment whatever the lane mask (out-of-range offsets drop the rest), so the loop's
      // counted vmcnt knows exactly how many stores follow the row's DMA
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), hrs,
                                             q < 3 && p < C::SW && c < W ? ((r * W + c) * 12 + 4 * q) * 4 : OOB_INL, 0, 0);
    }
  };

  auto conv2 = [&](int r) __attribute__((always_inline)) {
    // fragment addresses: pixel x = fp*16 + col + dw of ring row slot (r-1+dh) & 3, chunk q; swz2's pattern does not
    // depend on the slot (RW % 8 == 0), and fp = 1 is fp = 0 shifted by 16 pixels: +1024 bytes, the same swizzle
    // ((p + 16) >> 1) & 3 == (p >> 1) & 3
    int so[3], sx[3];
    {
      int l = lane;
      asm volatile("" : "+v"(l));
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) sx[dw] = swz2((l & 15) + dw, l >> 4);
    }
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) so[dh] = ((r - 1 + dh) & 3) * (C::RW * 64);
    f32x4 acc[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) acc[f][fp] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto frags = [&](uint4 (&bv)[2], int s) __attribute__((always_inline)) {
      const int g = s / 9, tap = s % 9;
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
        bv[fp] = *reinterpret_cast<const uint4*>(smem + g * C::PLANE + fp * 1024 + so[tap / 3] + sx[tap % 3]);
    };
    uint4 bv[2][2];
    frags(bv[0], 0);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      if (s + 1 < 18) frags(bv[(s + 1) & 1], s + 1);
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int fp = 0; fp < 2; ++fp) {
          if constexpr (ABL & 2) asm volatile("" ::"v"(bv[s & 1][fp].x), "v"(w2[s][f].x));
          else mma16<T>(w2[s][f], bv[s & 1][fp], acc[f][fp]);
        }
    }
    // pin the order: step s+1's 2 reads ahead of step s's 4 MFMAs
    if constexpr (PIN) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        if (s + 1 < 18) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
      }
    }

    if constexpr ((ABL & 16) != 0) {
      asm volatile("" ::"v"(acc[0][0][0]), "v"(acc[0][1][0]), "v"(acc[1][0][0]), "v"(acc[1][1][0]));
      return;
    }
    // epilogue: bias / affine / act in registers (lane-derived values recomputed from an opaque lane id, as in conv1)
    int l = lane;
    asm volatile("" : "+v"(l));
    const int cl = l & 15, ql = l >> 4;
    const int cq16 = (ql & 1) ? 2 + (ql >> 1) : ql >> 1;  // chunk_pair: the 16-byte chunk this lane ends up holding
    float mul[2][4], add[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float4 m4 = *reinterpret_cast<const float4*>(rk + 32 * wave + 16 * f + 4 * ql);
      const float4 a4 = *reinterpret_cast<const float4*>(rk + 64 + 32 * wave + 16 * f + 4 * ql);
      mul[f][0] = m4.x; mul[f][1] = m4.y; mul[f][2] = m4.z; mul[f][3] = m4.w;
      add[f][0] = a4.x; add[f][1] = a4.y; add[f][2] = a4.z; add[f][3] = a4.w;
    }
    const bool podd = (r & 1) != 0;
    const bool full = c0 + C::SW <= W;  // every stored column of the strip is inside the frame (uniform)
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) {
      const int c = c0 + fp * 16 + cl;
      const bool cok = fp * 16 + cl < C::SW && c < W;
      float v[2][4];
      uint2 pk[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = fmaf(acc[f][fp][j], mul[f][j], add[f][j]);
          if constexpr (ACT == VM_ACT_RELU) t = fmaxf(t, 0.f);
          else if constexpr (ACT == VM_ACT_SIGMOID) t = sigmoid_precise(t);
          v[f][j] = t;
        }
        pk[f].x = bf16x2_bits(v[f][0], v[f][1]);
        pk[f].y = bf16x2_bits(v[f][2], v[f][3]);
      }
      if (!a.y_skip) {
        const uint4 d = chunk_pair(pk[0], pk[1]);
        const int off = cok ? ((int)__umul24(r * W + c, ycs2) + (32 * wave + 8 * cq16) * 2) : OOB_INL;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                               off, 0, 0);
      }
      if (a.hd) {
        const uint4 hb = make_uint4(pk[0].x, pk[0].y, pk[1].x, pk[1].y);
        *reinterpret_cast<uint4*>(smem + C::X_OFF + ((((r & 1) * 2 + wave) * 2 + fp) * 64 + l) * 16) = hb;
      }
      if (a.py) {
        // fused 2x2 SAME max-pool: even rows wait in registers for their partner (rows past the frame never win);
        // the column partner is lane cl ^ 1 (DPP quad_perm [1,0,3,2]); bf16 rounding is monotonic, so the max of
        // the rounded values is the rounded max
        if (!podd && r + 1 < H) {
          prev[fp][0] = pk[0];
          prev[fp][1] = pk[1];
        } else {
          uint2 m2[2];
          if constexpr (ACT == VM_ACT_RELU) {
            // relu outputs are +0 or positive (never -0: the sum starts at +0 and the bias add cannot make -0 unless
            // the affine shift is -0), so the order of their bf16 bit patterns is the unsigned order: the pool runs
            // on the packed pairs (v_pk_max_u16), and a position outside the frame enters as 0, which never wins
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              uint32_t m[2] = {pk[f].x, pk[f].y};
              const uint32_t pp[2] = {prev[fp][f].x, prev[fp][f].y};
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                if (podd) m[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(
                                     __builtin_bit_cast(u16x2, m[h]), __builtin_bit_cast(u16x2, pp[h])));
                if (!full) m[h] = cok ? m[h] : 0u;
                const uint32_t u = (uint32_t)__builtin_amdgcn_mov_dpp((int)m[h], 0xB1, 0xF, 0xF, false);
                m[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, m[h]),
                                                                             __builtin_bit_cast(u16x2, u)));
              }
              m2[f] = make_uint2(m[0], m[1]);
            }
          } else {
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            float m[4];
            const uint2 pp = prev[fp][f];
            const float pv[4] = {__uint_as_float(pp.x << 16), __uint_as_float(pp.x & 0xffff0000u),
                                 __uint_as_float(pp.y << 16), __uint_as_float(pp.y & 0xffff0000u)};
            const float cv[4] = {__uint_as_float(pk[f].x << 16), __uint_as_float(pk[f].x & 0xffff0000u),
                                 __uint_as_float(pk[f].y << 16), __uint_as_float(pk[f].y & 0xffff0000u)};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float t = podd ? fmaxf(pv[j], cv[j]) : cv[j];
              t = cok ? t : -INFINITY;
              const float u = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xB1, 0xF, 0xF, false));
              m[j] = fmaxf(t, u);
            }
            m2[f].x = bf16x2_bits(m[0], m[1]);
            m2[f].y = bf16x2_bits(m[2], m[3]);
          }
          }
          const uint4 d = chunk_pair(m2[0], m2[1]);
          const int pr = r >> 1, pc = c >> 1;
          const bool pok = (cl & 1) == 0 && cok && pc < PWd;
          const int off = pok ? ((int)__umul24(pr * PWd + pc, a.py_cstride) + 32 * wave + 8 * cq16) * 2 : OOB_INL;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                 prs, off, 0, 0);
        }
      }
    }
  };

  // ---- warm-up: input rows s0-2 .. s0+3 through the staging ring two at a time, row s0+4 left in staging (converted
  // in the first iteration), then conv1_1 rows s0-1 .. s0+1
  for (int k = 0; k < 6; k += 2) {
    if (wave == 0) {
      dma_row(s0 - 2 + k, 0);
      dma_row(s0 - 1 + k, 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (wave == 0) {
      convert_row(s0 - 2 + k, 0);
      convert_row(s0 - 1 + k, 1);
    }
    __syncthreads();
  }
  if (wave == 0) {
    dma_row(s0 + 4, (s0 - 1) & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  conv1(s0 - 1);
  conv1(s0);
  conv1(s0 + 1);
  __syncthreads();

  for (int r = s0; r < s1; ++r) {
    int nst = 0;  // wave 0: vector-memory ops issued after this row's DMA (counted vmcnt before the barrier)
    if (wave == 0) {
      if constexpr (!(ABL & 8)) convert_row(r + 4, (r - 1) & 1);  // read from iteration r + 1 on, after the barrier
      if constexpr (!(ABL & 8)) dma_row(r + 5, r & 1);
      // the previous row's head partials after the DMA (r04): the barrier's counted wait then leaves them in flight
      // (issued before the DMA, in-order counting made every row wait for their write-back too)
      const bool hf = a.hd && r > s0;
      if (hf) head_finish(r - 1);
      nst = (hf ? 2 : 0) + (a.y_skip ? 0 : 2) + (a.py && ((r & 1) || r + 1 == H) ? 2 : 0);
    }
    conv1(r + 2);  // (row s1 + 1 at a segment's last row: computed into a ring slot nothing reads)
    conv2(r);
    if (wave == 0) {  // nst is 0, 2, 4 or 6
      if ((ABL & 8) || nst == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (nst == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (nst == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS-only barrier: global stores stay in flight
    if constexpr (!(ABL & 4)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (a.hd && wave == 0) head_finish(s1 - 1);
}

bool pair_strip_ok(const ConvArgs& a) {
  // the input window (36 pixels) is fetched whole by <= 2 LDS-DMA instructions and addressed with 32-bit offsets
  // (and an image holds at least the 2 KB a row fetch may span)
  const int es = a.x_f32 ? 4 : 2;
  const long imgb = (long)a.H * a.W * a.x_cstride * es;
  // (pixel indices of a frame < 2^24: the output offsets use the full-rate 24-bit multiply)
  return a.cout == 64 && a.x_c <= 8 && (a.x_f32 ? a.x_cstride <= 8 : a.x_cstride == 8) && imgb < 0x7ffffff0L - 4096 &&
         imgb >= 2048 && a.W > 0 && a.H > 0 && (long)a.H * a.W < (1L << 24);
}

long g_pair_strip_abl = 0;  // study build: timing-only ablations (1 no conv1_1 MFMAs, 2 no conv1_2 MFMAs, 4 no row
                            // barrier, 8 no input DMA, 16 no conv1_2 epilogue; garbage results)

long g_pair_strip_pin = 1;  // 1: conv1_2's LDS reads pinned 2 ahead of its MFMAs; 0: left to the scheduler (A/B)

template <int ACT, int ABL, int PIN = 1>
static void launch_strip_act(ConvArgs& a, long grid, int seg, int nseg, int nstrip, hipStream_t st) {
  if constexpr (PIN) {
    if (!g_pair_strip_pin) return launch_strip_act<ACT, ABL, 0>(a, grid, seg, nseg, nstrip, st);
  }
  if (a.x_f32 && a.x_c == 7)
    hipLaunchKernelGGL((conv3x3_pair_strip<2, ACT, ABL, PIN, 7>), dim3((unsigned)grid), dim3(128), StripCfg::LDS, st, a,
                       seg, nseg, nstrip);
  else if (a.x_f32)
    hipLaunchKernelGGL((conv3x3_pair_strip<2, ACT, ABL, PIN>), dim3((unsigned)grid), dim3(128), StripCfg::LDS, st, a, seg,
                       nseg, nstrip);
  else
    hipLaunchKernelGGL((conv3x3_pair_strip<0, ACT, ABL, PIN>), dim3((unsigned)grid), dim3(128), StripCfg::LDS, st, a, seg,
                       nseg, nstrip);
}
template <int ABL>
static void launch_strip_abl(ConvArgs& a, long grid, int seg, int nseg, int nstrip, hipStream_t st) {
  launch_strip_act<VM_ACT_RELU, ABL>(a, grid, seg, nseg, nstrip, st);
}

int launch_pair_strip(ConvArgs& a, long nimg, hipStream_t st) {
  static int attr_dev = -1, n_cu = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (attr_dev != dev) {
    hipError_t e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "conv3x3_pair_strip setup: %s", hipGetErrorString(e));
    attr_dev = dev;
  }
  // one round of 4 workgroups per CU: segments of equal (even) height so that images x segments x strips fills it
  const int nstrip = (a.W + StripCfg::SW - 1) / StripCfg::SW;
  const long slots = 4L * n_cu;
  long nseg = slots / (nimg * nstrip);
  if (nseg < 1) nseg = 1;
  int seg = (int)((a.H + nseg - 1) / nseg);
  seg += seg & 1;
  if (seg < 2) seg = 2;
  nseg = (a.H + seg - 1) / seg;
  const long grid = nimg * nseg * nstrip;
  if (grid > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_pair_strip: grid too large");
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_pair_strip");
#ifdef VM_STUDY
  switch (g_pair_strip_abl) {
    case 1: launch_strip_abl<1>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 2: launch_strip_abl<2>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 3: launch_strip_abl<3>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 4: launch_strip_abl<4>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 8: launch_strip_abl<8>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 16: launch_strip_abl<16>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 28: launch_strip_abl<28>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    case 31: launch_strip_abl<31>(a, grid, seg, (int)nseg, nstrip, st); return check_launch("abl");
    default: break;
  }
#endif
  switch (a.act) {
    case VM_ACT_RELU: launch_strip_act<VM_ACT_RELU, 0>(a, grid, seg, (int)nseg, nstrip, st); break;
    case VM_ACT_SIGMOID: launch_strip_act<VM_ACT_SIGMOID, 0>(a, grid, seg, (int)nseg, nstrip, st); break;
    default: launch_strip_act<VM_ACT_NONE, 0>(a, grid, seg, (int)nseg, nstrip, st); break;
  }
  return check_launch("conv3x3_pair_strip");
}

}  // namespace vm
