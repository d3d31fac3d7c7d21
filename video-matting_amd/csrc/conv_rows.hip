// 3x3 SAME conv with row-stationary register reuse (bf16 MFMA), the UNetVideo workhorse for large grids.
//
// Replaces tf.nn.conv2d + bias_add (+ relu / inference BN affine, + the fused 2x2 SAME max-pool of unet.py:32-33,
// + the folded 2x legacy resize of upconv_concat) at unet.py:35-42, 44-63 — the same math as conv3x3_patch, with a
// different wave tiling:
//
//   block  = persistent, one per CU, 8 waves (2 per SIMD); it walks a list of TH x 32 pixel x 64 channel tiles
//   wave   = R = 4 consecutive output rows x 32 pixels x CW output channels (TH 16: CW = 32)
//   K step = one 32-channel granule, all 9 taps: the (TH+2) x 34 input patch and the 9 x 64 weight rows are DMA'd
//            into LDS once per granule (double-buffered, buffer_load ... lds).
//
// Inside a granule every wave keeps the 9 taps' weight fragments of its channels in registers and walks its R+2
// input rows once: the pixel fragments of input row ir (3 horizontal shifts x 2 fragments) feed the MFMAs of every
// output row o = ir - kh they touch (up to 3 kernel rows).  Per MFMA a wave reads 0.375 KB of fragments from LDS
// (weights 18 + pixels 36 fragments per 144 MFMAs) where the 1-row x 64-channel waves of conv3x3_patch read 0.75 KB —
// the LDS-read budget that capped that kernel.
//
// Pipeline per granule g (two raw s_barriers, counted vmcnt, no __syncthreads in the loop):
//   rows 0..R-1 of g                      weights W(g) in registers, patch X(g)
//   B(g+1):  W(g+1) landed (vmcnt leaves X(g+1) in flight) -> DMA W(g+2) into W(g)'s buffer
//   rows R, R+1 of g; meanwhile W(g+1)'s kernel rows kh = 0, 1, 2 are read into the registers kh stops using
//            (kh 0 is dead after input row R-1, kh 1 after R, kh 2 after R+1)
//   B'(g+1): X(g+1) landed (vmcnt leaves W(g+2) in flight) -> DMA X(g+2) into X(g)'s buffer
// so each DMA has one granule to land and no wave waits on a fragment read right after a barrier.  The granule stream
// runs on across the block's tiles (the next tile's first granules are in flight while the last ones of this tile
// compute), and the epilogue works from registers (bias / affine / act, 8-byte stores, the 2x2 max-pool through a
// lane exchange), so a tile change costs no LDS round trip, no block-wide barrier and no DMA latency.
#include <type_traits>

#include "conv_common.h"

namespace vm {

template <int TH_>
struct RowsCfg {
  static constexpr int R = 4;                          // output rows per wave
  static constexpr int TH = TH_, TW = 32, BM = TH * TW, BN = 64;
  static constexpr int RG = TH / R, CG = 8 / RG;       // wave grid: row groups x channel groups (8 waves)
  static constexpr int CW = BN / CG, FC = CW / 16;     // channels / 16-channel fragments per wave
  static constexpr int PW = TW + 2, PPIX = (TH + 2) * PW;
  static constexpr int XP = (PPIX + 15) / 16, XPW = (XP + 7) / 8;  // patch DMA pieces (16 LDS rows each)
  static constexpr int PB = XP * 1024;
  static constexpr int WP = 9 * BN / 16, WPW = (WP + 7) / 8;       // weight DMA pieces per granule
  static constexpr int WB = 9 * BN * 64;               // 9 tap slots of 64 rows x 64 B
  static constexpr int JUNK = 2 * PB + 2 * WB;          // 1 KiB landing slot of the padding DMA pieces
  static constexpr int LDS = JUNK + 1024;
  static_assert(RG * CG == 8 && FC >= 1, "8 waves");
  static_assert(LDS <= 163840, "one CU's LDS");
};

// MFMAs fed by input row ir (0..5) of a 4-row wave: kernel rows kh with 0 <= ir - kh < 4, x 3 taps x FC x 2
template <int FC>
constexpr int row_mfmas(int ir) {
  int k = 0;
  for (int kh = 0; kh < 3; ++kh) k += (ir - kh >= 0 && ir - kh < 4) ? 1 : 0;
  return k * 3 * FC * 2;
}

// sched_group_barrier sequence: M MFMAs with D LDS reads spread evenly among them (each read after M/D MFMAs)
template <int M, int D>
__device__ __forceinline__ void sched_spread() {
  constexpr int per = D ? M / D : M;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, per, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
  if constexpr (M - per * D > 0) __builtin_amdgcn_sched_group_barrier(0x008, M - per * D, 0);
}

// rows 0..3 of a granule: D0 reads up front (input rows 0, 1), then row r's MFMAs with row r+2's reads spread in
template <int FC, int D0, int D1, int D2, int D3, int D4>
__device__ __forceinline__ void sched_rows() {
  __builtin_amdgcn_sched_group_barrier(0x100, D0, 0);
  sched_spread<row_mfmas<FC>(0), D1>();
  sched_spread<row_mfmas<FC>(1), D2>();
  sched_spread<row_mfmas<FC>(2), D3>();
  sched_spread<row_mfmas<FC>(3), D4>();
}

// rows 4, 5: input row 5 + the next granule's kernel rows 0 and 2 under row 4, its kernel row 1 under row 5
template <int FC>
__device__ __forceinline__ void sched_tail() {
  sched_spread<row_mfmas<FC>(4), 6 + 6 * FC>();
  sched_spread<row_mfmas<FC>(5), 3 * FC>();
}

struct RowTile {
  int n, r0, c0, n0;
};

// split-fp16 x3 output of 4 channels: h = fp16(v), l = fp16(v - h) as two 8-byte quads; true if some |v| >= 65520
__device__ __forceinline__ bool split4h(const float (&v)[4], uint2& h, uint2& l) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t a = {v[0], v[1]}, b = {v[2], v[3]};
  const h2_t ha = __builtin_convertvector(a, h2_t), hb = __builtin_convertvector(b, h2_t);
  const f2_t ra = {v[0] - (float)ha[0], v[1] - (float)ha[1]}, rb = {v[2] - (float)hb[0], v[3] - (float)hb[1]};
  h = make_uint2(__builtin_bit_cast(uint32_t, ha), __builtin_bit_cast(uint32_t, hb));
  l = make_uint2(__builtin_bit_cast(uint32_t, __builtin_convertvector(ra, h2_t)),
                 __builtin_bit_cast(uint32_t, __builtin_convertvector(rb, h2_t)));
  return !(fabsf(v[0]) < 65520.f) || !(fabsf(v[1]) < 65520.f) || !(fabsf(v[2]) < 65520.f) || !(fabsf(v[3]) < 65520.f);
}

// SPL: the split-fp16 x3 form (vmatting/split3.py): fp16 operands (v_mfma_f32_16x16x32_f16) and the output written
// split as [l, h(, h)] slabs (ConvArgs::ysplit / psplit / ovf) from the same register epilogue
template <int TH, bool SPL = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void conv3x3_rows(ConvArgs a) {
  using C = RowsCfg<TH>;
  using T = uint16_t;
  using MT = std::conditional_t<SPL, f16_t, uint16_t>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int R = C::R, FC = C::FC, XPW = C::XPW, WPW = C::WPW, PW = C::PW;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int rg = wave % C::RG, cg = wave / C::RG;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + C::TW - 1) / C::TW;

  // this block's tiles: XCD x = blockIdx.x % 8 owns the contiguous eighth [lo, hi) of the tile list (the 64-channel
  // slices of one patch and the neighbouring patches share that XCD's L2); its gridDim.x / 8 blocks take every
  // nslot-th tile of it
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int lo = (int)((long)xcd * a.tiles_total / 8), hi = (int)((long)(xcd + 1) * a.tiles_total / 8);
  const int ntile = slot < hi - lo ? (hi - lo - slot + nslot - 1) / nslot : 0;
  const int nch = a.cin_pad / 32;
  const int S = ntile * nch;  // granule steps of this block
  if (S == 0) return;
  auto tile_of = [&](int k) __attribute__((always_inline)) {
    const int t = lo + slot + k * nslot;
    const int st = t / a.tiles_n, nt = t - st * a.tiles_n;  // consecutive tiles: the same patch, next 64 channels
    RowTile r;
    r.n = st / (th * tw);
    const int srem = st - r.n * th * tw;
    r.r0 = (srem / tw) * TH;
    r.c0 = (srem - (srem / tw) * tw) * C::TW;
    r.n0 = nt * C::BN;
    // wave-uniform by construction; say so, so buffer descriptors built from it stay in SGPRs
    r.n = __builtin_amdgcn_readfirstlane(r.n);
    r.r0 = __builtin_amdgcn_readfirstlane(r.r0);
    r.c0 = __builtin_amdgcn_readfirstlane(r.c0);
    r.n0 = __builtin_amdgcn_readfirstlane(r.n0);
    return r;
  };

  // DMA geometry (as conv3x3_patch): piece k fills 16 LDS rows of 64 B; the lane filling physical chunk lpos of row r
  // fetches logical chunk swz(r, lpos); SAME padding / rows past the patch get an out-of-range offset (zeros).
  // Tile-independent per-lane part packed as (patch row << 16) | (patch column << 8) | logical chunk.
  const int lrow = lane >> 2, lpos = lane & 3;
  int xgeo[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int piece = wave + i * 8;
    const int row = piece * 16 + lrow;
    const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
    const int pr = row / PW, pc = row - pr * PW;
    xgeo[i] = row < C::PPIX ? (pr << 16) | (pc << 8) | lq : -1;
  }
  int woff[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int piece = wave + i * 8;
    const int tap = piece / (C::BN / 16);
    const int row = (piece - tap * (C::BN / 16)) * 16 + lrow;  // output channel inside the tap slot
    const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
    woff[i] = (row * a.K_pad + lq * 8) * 2 + tap * 64;           // chunk-major K: granule cc*9 + tap
  }
  // LDS: weight buffers [0, 2 WB), patch buffers [2 WB, 2 WB + 2 PB)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  // per-channel epilogue constants (mul, add) of every output channel, staged in LDS once per block (r04): read from
  // global memory inside the epilogue they made hipcc wait vmcnt(0) there, draining the next granules' DMA at every
  // tile end; published by the prologue's barrier
  const int ccap = a.up ? a.up_cout : a.cout;
  float2* const ctab = reinterpret_cast<float2*>(smem + C::LDS);
  for (int c = tid; c < ccap; c += 512) {
    const float sc = a.scale ? a.scale[c] : 1.f;
    ctab[c] = make_float2(sc, (a.bias ? a.bias[c] : 0.f) * sc + (a.shift ? a.shift[c] : 0.f));
  }
  // DMA of granule g of local tile k into buffer buf; k >= ntile issues the same number of out-of-range (zero) pieces,
  // so every wave's vmcnt bookkeeping stays uniform
  // DMA of granule g of tile tt into buffer buf.  Every wave issues exactly XPW patch and WPW weight pieces (pieces past
  // the patch / weight slot land in the junk slot), so the vmcnt counts below are compile-time constants; real ==
  // false (steps past the end) turns every piece into an out-of-range (zero) load with the same count.
  auto issue_x = [&](const RowTile& tt, bool real, int g, int buf, auto i0c, auto i1c) __attribute__((always_inline)) {
    constexpr int i0 = decltype(i0c)::value, i1 = decltype(i1c)::value;
    const T* xb = uniform_ptr(reinterpret_cast<const T*>(a.x) + a.x_coff + (long)tt.n * H * W * cs);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xb), 0, 0x7ffffff0, 0x00020000);
    const int coff = (int)src_chan(a, g * 32) * 2;
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const bool piece_ok = wave + i * 8 < C::XP;
      int h = tt.r0 - 1 + (xgeo[i] >> 16), w = tt.c0 - 1 + ((xgeo[i] >> 8) & 255);
      if (a.up) {  // folded 2x resize: past the bottom/right edge the low-res frame is replicated (TF1 clamp)
        h = min(h, H - 1);
        w = min(w, W - 1);
      }
      const bool ok = real && xgeo[i] >= 0 && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      glds16(xrs, __builtin_amdgcn_readfirstlane(lds0 + (piece_ok ? 2 * C::WB + buf * C::PB + (wave + i * 8) * 1024 : C::JUNK)),
             ok ? ((h * W + w) * cs + (xgeo[i] & 255) * 8) * 2 + coff : OOB);
    }
  };
  auto issue_w = [&](int n0, bool real, int g, int buf, auto i0c, auto i1c) __attribute__((always_inline)) {
    constexpr int i0 = decltype(i0c)::value, i1 = decltype(i1c)::value;
    const T* wb = uniform_ptr(reinterpret_cast<const T*>(a.w) + (long)n0 * a.K_pad);
    const uint32_t wbytes = __builtin_amdgcn_readfirstlane((uint32_t)((long)(a.cout_pad - n0) * a.K_pad * 2));
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(wb), 0, wbytes, 0x00020000);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const bool piece_ok = wave + i * 8 < C::WP;
      glds16(wrs, __builtin_amdgcn_readfirstlane(lds0 + (piece_ok ? buf * C::WB + (wave + i * 8) * 1024 : C::JUNK)),
             real && piece_ok ? woff[i] + g * 576 : OOB);
    }
  };
  // raw barrier after a counted DMA wait; lgkmcnt(0) retires this wave's fragment reads of the buffer the DMA
  // issued right after the barrier refills (the MFMAs consuming them may be scheduled past the barrier)
  auto sync = [&](auto nconst) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(nconst)::value) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // fragment addresses: per-lane VGPR bases + compile-time offsets (ds_read_b128 offset field).
  // Pixel fragment (input row ir, pixel half pf, tap column kw) is patch row p = pbase + K, K = ir*PW + pf*16 + kw;
  // swz<64> flips chunk bit 1 by bit 2 of p, which is bit 2 of (pbase % 8 + K % 8): one base per K % 8.
  const int ck = lane >> 4, col = lane & 15;
  const int pbase = rg * R * PW + col;
  int pxa[8];
#pragma unroll
  for (int v = 0; v < 8; ++v)
    pxa[v] = 2 * C::WB + pbase * 64 + ((ck ^ ((((pbase & 7) + v) >> 2) & 1) * 2) << 4);
  int wa[FC];
#pragma unroll
  for (int f = 0; f < FC; ++f) wa[f] = swz<64>(cg * C::CW + f * 16 + col, ck);

  typedef uint4 WRow[3][FC];  // one kernel row: 3 taps x FC channel fragments
  auto ldw = [&](WRow& w, const int buf, const int kh) __attribute__((always_inline)) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int f = 0; f < FC; ++f)
        w[kw][f] = *reinterpret_cast<const uint4*>(smem + wa[f] + buf * C::WB + (kh * 3 + kw) * (C::BN * 64));
  };
  typedef uint4 XRow[3][2];  // one input row: 3 tap columns x 2 pixel fragments
  auto ldx = [&](XRow& x, const int buf, const int ir) __attribute__((always_inline)) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int pf = 0; pf < 2; ++pf) {
        const int K = ir * PW + pf * 16 + kw;
        x[kw][pf] = *reinterpret_cast<const uint4*>(smem + pxa[K & 7] + K * 64 + buf * C::PB);
      }
  };

  f32x4 acc[R][FC][2];
#pragma unroll
  for (int o = 0; o < R; ++o)
#pragma unroll
    for (int f = 0; f < FC; ++f)
#pragma unroll
      for (int pf = 0; pf < 2; ++pf) acc[o][f][pf] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight registers: kernel rows 0 and 1 are reloaded in place; kernel row 2 alternates between w2 (even steps)
  // and w3 (odd steps), so the next granule's row 2 is read while this granule's row 2 still feeds MFMAs
  WRow w0, w1, w2, w3;
  // input row ir of the wave's (R+2)-row window: MFMAs into every output row it reaches (ir is a compile-time
  // constant after unrolling, so the kernel-row selection folds away)
  auto row_mma = [&](const int ir, const XRow& x, const WRow& k2) __attribute__((always_inline)) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int o = ir - kh;
        if (o < 0 || o >= R) continue;
#pragma unroll
        for (int f = 0; f < FC; ++f)
#pragma unroll
          for (int pf = 0; pf < 2; ++pf) {
            const uint4& wv = kh == 0 ? w0[kw][f] : (kh == 1 ? w1[kw][f] : k2[kw][f]);
            mma16<MT>(wv, x[kw][pf], acc[o][f][pf]);
          }
      }
  };

  // epilogue of tile tt from the accumulators: lane (ck, col) holds channels chn..chn+3 (chn = cg*CW + f*16 + 4*ck)
  // of pixel (r0 + rg*R + o, c0 + pf*16 + col).  bias / inference-BN affine / act, bf16, one 8-byte store each;
  // a.up scatters phase (n0 / up_cout) to pixel (2h + p/2, 2w + p%2); a.py gets the 2x2 SAME max-pool (rows o, o+1
  // in this lane, columns col, col+1 in the neighbouring lane; positions past the frame never win)
  bool ovf = false;  // SPL: some output left fp16's range
  auto epilogue = [&](const RowTile& tt) __attribute__((always_inline)) {
    const int phase = a.up ? tt.n0 / a.up_cout : 0;
    const int cb = tt.n0 - phase * a.up_cout;  // first (per-phase) output channel of the tile
    const int YH = a.up ? 2 * H : H, YW = a.up ? 2 * W : W;
    T* yb = uniform_ptr(reinterpret_cast<T*>(a.y) + a.y_coff + (long)tt.n * YH * YW * a.y_cstride);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yb, 0, 0x7ffffff0, 0x00020000);
    const int PH = (H + 1) >> 1, PWo = (W + 1) >> 1;
    T* pbp = uniform_ptr(a.py ? reinterpret_cast<T*>(a.py) + a.py_coff + (long)tt.n * PH * PWo * a.py_cstride : nullptr);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pbp, 0, 0x7ffffff0, 0x00020000);
    float mul[FC][4], add[FC][4];
#pragma unroll
    for (int f = 0; f < FC; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 t = ctab[min(cb + cg * C::CW + f * 16 + 4 * ck + j, ccap - 1)];
        mul[f][j] = t.x;
        add[f][j] = t.y;
      }
    auto pack4 = [](const float (&v)[4]) __attribute__((always_inline)) {
      return make_uint2(bf16x2_bits(v[0], v[1]), bf16x2_bits(v[2], v[3]));
    };
    // FC == 2: the two 16-channel fragments form one 32-channel group, and chunk_pair turns the lanes' 4-channel quads
    // into whole 16-byte chunks (chunk c16 of the group): one 16-byte store per pixel row instead of two 8-byte ones
    const int c16 = (ck & 1) ? 2 + (ck >> 1) : ck >> 1;
#pragma unroll
    for (int pf = 0; pf < 2; ++pf) {
      const int c = tt.c0 + pf * 16 + col;
      float v[R][FC][4];
#pragma unroll
      for (int o = 0; o < R; ++o) {
        const int r = tt.r0 + rg * R + o;
#pragma unroll
        for (int f = 0; f < FC; ++f)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float t = fmaf(acc[o][f][pf][j], mul[f][j], add[f][j]);
            if (a.act == VM_ACT_RELU) t = fmaxf(t, 0.f);
            else if (a.act == VM_ACT_SIGMOID) t = sigmoid_precise(t);
            v[o][f][j] = t;
          }
        const int pix = a.up ? (2 * r + (phase >> 1)) * YW + 2 * c + (phase & 1) : r * W + c;
        if constexpr (SPL) {  // [l, h(, h)]: slab distance ysplit, the third where the pixel row holds it
          typedef __attribute__((ext_vector_type(4))) unsigned u4_t;
          typedef __attribute__((ext_vector_type(2))) unsigned u2_t;
          const int S2 = a.ysplit * 2;
          const bool y3 = 3 * a.ysplit <= a.y_cstride;
          uint2 hq[FC], lq[FC];
          bool o2 = false;
#pragma unroll
          for (int f = 0; f < FC; ++f) o2 |= split4h(v[o][f], hq[f], lq[f]);
          if constexpr (FC == 2) {
            const int chan = cb + cg * C::CW + c16 * 8;
            const bool ok = r < H && c < W && chan < ccap;
            ovf |= ok && o2;
            const int off = ok ? (pix * a.y_cstride + chan) * 2 : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, chunk_pair(lq[0], lq[1])), yrs, off, 0, 0);
            const uint4 dh = chunk_pair(hq[0], hq[1]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, dh), yrs, ok ? off + S2 : OOB, 0, 0);
            if (y3) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, dh), yrs, ok ? off + 2 * S2 : OOB, 0, 0);
          } else {
#pragma unroll
            for (int f = 0; f < FC; ++f) {
              const int chan = cb + cg * C::CW + f * 16 + 4 * ck;
              const bool ok = r < H && c < W && chan < ccap;
              ovf |= ok && o2;
              const int off = ok ? (pix * a.y_cstride + chan) * 2 : OOB;
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, lq[f]), yrs, off, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, hq[f]), yrs, ok ? off + S2 : OOB, 0, 0);
              if (y3) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, hq[f]), yrs, ok ? off + 2 * S2 : OOB, 0, 0);
            }
          }
        } else if constexpr (FC == 2) {
          const int chan = cb + cg * C::CW + c16 * 8;
          const uint4 d = chunk_pair(pack4(v[o][0]), pack4(v[o][1]));
          const bool ok = r < H && c < W && chan < ccap;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                 yrs, ok ? (pix * a.y_cstride + chan) * 2 : OOB, 0, 0);
        } else {
#pragma unroll
          for (int f = 0; f < FC; ++f) {
            const int chan = cb + cg * C::CW + f * 16 + 4 * ck;
            const bool ok = r < H && c < W && chan < ccap;
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, pack4(v[o][f])), yrs,
                ok ? (pix * a.y_cstride + chan) * 2 : OOB, 0, 0);
          }
        }
      }
      if (a.py) {
#pragma unroll
        for (int op = 0; op < R / 2; ++op) {
          const int r = tt.r0 + rg * R + 2 * op;  // even: the window's top row
          const bool v0 = r < H && c < W, v1 = r + 1 < H && c < W;
          float m[FC][4];
#pragma unroll
          for (int f = 0; f < FC; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float t = v0 ? v[2 * op][f][j] : -INFINITY;
              if (v1) t = fmaxf(t, v[2 * op + 1][f][j]);
              // column partner: lane col ^ 1 (DPP quad_perm [1,0,3,2])
              const float u = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xB1, 0xF, 0xF, false));
              m[f][j] = fmaxf(t, u);
            }
          const int pr = r >> 1, pc = c >> 1;
          const bool pok = (col & 1) == 0 && pr < PH && pc < PWo;
          if constexpr (SPL) {
            typedef __attribute__((ext_vector_type(4))) unsigned u4_t;
            typedef __attribute__((ext_vector_type(2))) unsigned u2_t;
            const int P2 = a.psplit * 2;
            const bool p3 = 3 * a.psplit <= a.py_cstride;
            uint2 hq[FC], lq[FC];
#pragma unroll
            for (int f = 0; f < FC; ++f) split4h(m[f], hq[f], lq[f]);
            if constexpr (FC == 2) {
              const int chan = tt.n0 + cg * C::CW + c16 * 8;
              const int off = pok && chan < a.cout ? ((pr * PWo + pc) * a.py_cstride + chan) * 2 : OOB;
              const uint4 dh = chunk_pair(hq[0], hq[1]);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, chunk_pair(lq[0], lq[1])), prs, off, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, dh), prs, off == OOB ? OOB : off + P2, 0, 0);
              if (p3)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, dh), prs, off == OOB ? OOB : off + 2 * P2, 0,
                                                       0);
            } else {
#pragma unroll
              for (int f = 0; f < FC; ++f) {
                const int chan = tt.n0 + cg * C::CW + f * 16 + 4 * ck;
                const int off = pok && chan < a.cout ? ((pr * PWo + pc) * a.py_cstride + chan) * 2 : OOB;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, lq[f]), prs, off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, hq[f]), prs, off == OOB ? OOB : off + P2, 0, 0);
                if (p3)
                  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, hq[f]), prs, off == OOB ? OOB : off + 2 * P2,
                                                        0, 0);
              }
            }
          } else if constexpr (FC == 2) {
            const int chan = tt.n0 + cg * C::CW + c16 * 8;
            const uint4 d = chunk_pair(pack4(m[0]), pack4(m[1]));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                   prs, pok && chan < a.cout ? ((pr * PWo + pc) * a.py_cstride + chan) * 2 : OOB,
                                                   0, 0);
          } else {
#pragma unroll
            for (int f = 0; f < FC; ++f) {
              const int chan = tt.n0 + cg * C::CW + f * 16 + 4 * ck;
              __builtin_amdgcn_raw_buffer_store_b64(
                  __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, pack4(m[f])), prs,
                  pok && chan < a.cout ? ((pr * PWo + pc) * a.py_cstride + chan) * 2 : OOB, 0, 0);
            }
          }
        }
      }
    }
  };

  // the step stream: step s = granule g of local tile k; t0 / t1 / t2 = tiles k, k+1, k+2 (decoded once per tile)
  int s = 0, k = 0, g = 0;
  RowTile t0 = tile_of(0), t1 = tile_of(ntile > 1 ? 1 : 0), t2 = tile_of(ntile > 2 ? 2 : 0);
  using Z = std::integral_constant<int, 0>;
  using NX = std::integral_constant<int, XPW>;
  using NW = std::integral_constant<int, WPW>;
  // DMA of step s + d (d = 1, 2): its tile is k + (g + d) / nch (at most k + 2).  Branch-free (scalar selects of
  // the candidate tiles' fields), so the pieces can sit among the MFMAs of one basic block; pieces [i0, i1) only
  auto issue_step = [&](int d, bool wts, int buf, auto i0, auto i1) __attribute__((always_inline)) {
    const int gd = g + d;
    const int dk = (gd >= nch ? 1 : 0) + (gd >= 2 * nch ? 1 : 0);
    const int gg = gd - dk * nch;
    // (arithmetic, not a select between the tile structs: that one demoted the register arrays to scratch)
    const int m1 = dk >= 1, m2 = dk >= 2;
    RowTile tt;
    tt.n = t0.n + m1 * (t1.n - t0.n) + m2 * (t2.n - t1.n);
    tt.r0 = t0.r0 + m1 * (t1.r0 - t0.r0) + m2 * (t2.r0 - t1.r0);
    tt.c0 = t0.c0 + m1 * (t1.c0 - t0.c0) + m2 * (t2.c0 - t1.c0);
    tt.n0 = t0.n0 + m1 * (t1.n0 - t0.n0) + m2 * (t2.n0 - t1.n0);
    const bool real = k + dk < ntile;
    if (wts) issue_w(tt.n0, real, gg, buf, i0, i1);
    else issue_x(tt, real, gg, buf, i0, i1);
  };
  // prologue: step 0 in, then step 1's DMA in flight
  using I = std::integral_constant<int, 0>;
  issue_w(t0.n0, true, 0, 0, I{}, NW{});
  issue_x(t0, true, 0, 0, I{}, NX{});
  sync(Z{});
  issue_step(1, true, 1, I{}, NW{});  // W(1); X(1) goes out at the start of step 0, among its MFMAs
  ldw(w0, 0, 0);
  ldw(w1, 0, 1);
  ldw(w2, 0, 2);

  // one step; b = s & 1 is a compile-time constant (the loop runs step pairs), so every fragment address is a
  // per-lane base + an immediate offset.  sched_group_barrier pins the interleave: the fragment reads of input row
  // ir+2 (and of the next granule's weights) are spread over row ir's MFMAs, so LDS latency stays hidden.
  auto step = [&](auto bconst) __attribute__((always_inline)) {
    constexpr int b = decltype(bconst)::value;
    static_assert(R == 4, "the row schedule below is written for 4-row waves");
    WRow& k2 = b == 0 ? w2 : w3;  // this step's kernel row 2
    WRow& n2 = b == 0 ? w3 : w2;  // the next step's
    XRow xa, xb;
    // X(s+1) into X(s-1)'s buffer (every wave retired its reads of it at B'(s)), its pieces among rows 0..2's MFMAs;
    // steps past the end issue the same number of zero pieces, so barriers and vmcnt counts stay uniform
    ldx(xa, b, 0);
    ldx(xb, b, 1);
    issue_step(1, false, b ^ 1, I{}, std::integral_constant<int, 2>{});
    row_mma(0, xa, k2);
    ldx(xa, b, 2);
    issue_step(1, false, b ^ 1, std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
    row_mma(1, xb, k2);
    ldx(xb, b, 3);
    issue_step(1, false, b ^ 1, std::integral_constant<int, 4>{}, NX{});
    row_mma(2, xa, k2);
    ldx(xa, b, 4);
    row_mma(3, xb, k2);
    sched_rows<FC, 12, 6, 6, 6, 0>();
    __builtin_amdgcn_sched_barrier(0);
    sync(NX{});  // B(s+1): W(s+1) landed, X(s+1) may still fly
    __builtin_amdgcn_sched_barrier(0);
    // W(s) lives in registers: its buffer takes W(s+2), pieces among rows 4, 5's MFMAs
    ldx(xb, b, 5);
    issue_step(2, true, b, I{}, std::integral_constant<int, 2>{});
    ldw(w0, b ^ 1, 0);  // kernel row 0 is dead after input row 3 (read anyway on the last step: unused)
    issue_step(2, true, b, std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
    ldw(n2, b ^ 1, 2);
    row_mma(4, xa, k2);
    issue_step(2, true, b, std::integral_constant<int, 4>{}, NW{});
    ldw(w1, b ^ 1, 1);  // kernel row 1 is dead after input row 4
    row_mma(5, xb, k2);
    sched_tail<FC>();
    __builtin_amdgcn_sched_barrier(0);
    sync(NW{});  // B'(s+1): X(s+1) landed, W(s+2) may still fly
    if (g == nch - 1) {  // last granule of the tile: write it out, restart the accumulators
      epilogue(t0);
#pragma unroll
      for (int o = 0; o < R; ++o)
#pragma unroll
        for (int f = 0; f < FC; ++f)
#pragma unroll
          for (int pf = 0; pf < 2; ++pf) acc[o][f][pf] = f32x4{0.f, 0.f, 0.f, 0.f};
      g = 0;
      ++k;
      t0 = t1;
      t1 = t2;
      if (k + 2 < ntile) t2 = tile_of(k + 2);
    } else {
      ++g;
    }
    ++s;
  };
  while (s < S) {
    step(std::integral_constant<int, 0>{});
    if (s < S) step(std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy DMAs past the end must land before the block exits
  if (SPL && ovf && a.ovf) *a.ovf = 1;  // a plain vector store: any writer's 1 is the answer
}

// the row-stationary kernel takes: bf16 in / bf16 out (16-byte aligned views), chunk-major 32-channel granules, no
// split-K, no softmax epilogue, 32-bit byte offsets inside one image (conv3x3_patch covers everything else)
bool rows_ok(const ConvArgs& a) {
  const long img_in = (long)a.H * a.W * a.x_cstride * 2;
  const long img_out = (long)(a.up ? 4 : 1) * a.H * a.W * a.y_cstride * 2;
  // (SPL: fp16 operands with the split output, ConvArgs::ysplit; plain f16 with an f32 output stays on the patch kernel)
  const bool yok = a.f16 ? a.ysplit > 0 : a.y_dtype == VM_BF16;
  return a.chunk_major && a.cin_pad % 32 == 0 && yok && a.y_vec && (a.cout & 7) == 0 &&
         a.act != VM_ACT_SOFTMAX && a.ksplit <= 1 && (a.x_src_c <= 0 || a.x_src_c % 32 == 0) &&
         (!a.up || a.up_cout % 64 == 0) && img_in < 0x7ffffff0L && img_out < 0x7ffffff0L &&
         (!a.py || (a.py_cstride % 8 == 0 && a.py_coff % 8 == 0)) &&
         RowsCfg<16>::LDS + 8 * (a.up ? a.up_cout : a.cout) <= 163840;  // + the epilogue constants table
}

static int g_num_cu = 0;

template <int TH, bool SPL>
static int launch_th(ConvArgs& a, hipStream_t st) {
  using C = RowsCfg<TH>;
  const int lds = C::LDS + 8 * (a.up ? a.up_cout : a.cout);  // + the epilogue constants table
  if (lds > 163840) return fail(VM_EUNSUPPORTED, "conv3x3_rows: %d output channels overflow LDS", a.cout);
  static bool attr_set = false;  // idempotent; benign race
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_rows<TH, SPL>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    if (e != hipSuccess) return fail(VM_EHIP, "hipFuncSetAttribute(rows): %s", hipGetErrorString(e));
    attr_set = true;
  }
  if (!g_num_cu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return fail(VM_EHIP, "conv3x3_rows: cannot read the CU count");
    g_num_cu = n;
  }
  const long N = a.M / ((long)a.H * a.W);
  const long sp = N * ((a.H + TH - 1) / TH) * ((a.W + C::TW - 1) / C::TW);
  a.tiles_n = (a.cout + C::BN - 1) / C::BN;
  if (sp * a.tiles_n > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3: too many tiles");
  a.tiles_total = (int)(sp * a.tiles_n);
  a.prio = (int)g_conv_prio;
  // persistent: one block per CU (LDS-limited), a multiple of 8 so every XCD gets the same number of blocks
  long grid = g_num_cu < a.tiles_total ? g_num_cu : a.tiles_total;
  grid = (grid + 7) / 8 * 8;
  snprintf(g_last_kernel, sizeof g_last_kernel, SPL ? "vm::conv3x3_rows<%d, true>" : "vm::conv3x3_rows<%d>", TH);
  hipLaunchKernelGGL((conv3x3_rows<TH, SPL>), dim3(grid), dim3(512), lds, st, a);
  return check_launch("conv3x3_rows");
}

// cfg: 16 or 8 = tile height (TH 8: 2 row groups x 4 channel groups of 16)
int launch_rows(ConvArgs& a, hipStream_t st, int cfg) {
  if (a.f16) {
    if (a.ysplit <= 0) return fail(VM_EUNSUPPORTED, "conv3x3_rows: fp16 operands need the split output");
    return cfg == 8 ? launch_th<8, true>(a, st) : launch_th<16, true>(a, st);
  }
  if (cfg == 8) return launch_th<8, false>(a, st);
  return launch_th<16, false>(a, st);
}

}  // namespace vm
