// Conv argument block and device helpers shared by the 3x3 conv kernels (conv3x3.hip, conv_rows.hip).
#pragma once

#include <type_traits>

#include "vm_common.h"

namespace vm {

struct ConvArgs {
  const void* x;
  int x_cstride, x_coff, H, W;
  long M;  // N*H*W pixels
  int cin_pad, K9, nk;
  int chunk_major, ng;  // granule layout and number of real granules (chunk-major)
  const void* w;
  int K_pad, cout, cout_pad;
  const float* bias;
  const float* scale;
  const float* shift;
  int act;
  void* y;
  int y_cstride, y_coff, y_dtype, y_vec;
  int tiles_n, tiles_total;
  void* py;  // optional fused 2x2/2 SAME max-pool output (patch kernel only), bf16 view
  int py_cstride, py_coff;
  int up, up_cout;  // folded 2x resize (patch kernel only): cout = 4 phases x up_cout, y is [N,2H,2W,up_cout]
  const void* w1;   // FIRST patch kernel: packed cin<=8 -> 64 first conv (tap-major, K_pad 128) and its bias
  const float* bias1;
  int x_f32, x_c;   // FIRST: the frame is f32 with x_c channels (converted to bf16 in the prologue)
  // x_src_c > 0: the input channels come from cin / x_src_c sources of x_src_c channels each, source s at
  // x_src_stride elements from the view base (tower-major features: unet_simple.py:153-168's concat, never built)
  int x_src_c;
  long x_src_stride;
  // split-K (patch kernel, row-slot pipeline): ksplit > 1 splits the channel granules over gridDim.y; each split
  // writes raw f32 sums to part[split][pixel][cout] and splitk_reduce_kernel applies bias/affine/act (fixed order)
  int ksplit;
  float* part;
  // pair kernel + head split (unet.py:203 conv1_5 over cat1 = [up, skip]): hd != nullptr makes the pair kernel also
  // write the skip half's per-tap head partials hd[pixel][12] (taps 0..8 of sum_c y[pixel][c] * hw[tap][hw_coff + c],
  // hw = the head's HWIO f32 filter with hw_cin input channels); y_skip = 1 leaves conv1_2's output unwritten
  float* hd;
  const float* hw;
  int hw_cin, hw_coff, y_skip;
  // packed frames (patch kernel): vstride > 0 tiles the batch as ONE virtual image of width vW = N * vstride whose
  // column v is column v % vstride of frame v / vstride; vstride = W + 2, so every frame is followed by two columns
  // outside it (zero input: the SAME padding of both neighbours; their outputs are never stored).  Narrow frames
  // (40 or 20 px in 32-px tiles) stop wasting most of their last column tile.
  int vstride, vW;
  int repi;  // patch kernel: 1 = register epilogue where the tiling allows (bf16 output, no split-K, no packed frames)
  int prot;  // persistent patch kernel: 1 = walkers rotate through the output tiles (folded-upconv phases)
  int upmask;  // folded upconvs: bit 0 = skip the zero kernel row, bit 1 = the zero kernel column (3 = both)
  // streaming patch kernel: cband > 0 maps block b to output tile (b & 7) * cband + (b >> 3) % cband of pixel tile
  // (b >> 3) / cband, so XCD b % 8 keeps its cband 64-channel weight slices L2-resident over every pixel tile (weight-
  // heavy layers: upconv_2's 9.4 MB folded filter, which the pixel-banded order re-streams per resident round)
  int cband;
  int ngroup;  // patch kernel: output-channel tiles per group of the tile order (0: all of a pixel tile's together)
  int twalk;  // conv3x3_thin: XCD-banded tile walk
  int seg;    // conv3x3_first_softmax_f32r: rows per wave segment
  int prio;  // 1: waves 4..7 of an 8-wave block run at s_setprio 1 (static priority for the arbitration loser)
  // strip pair kernel: optional bf16 output of the FIRST conv (conv1_1 + bias + relu), [N,H,W,64] view
  void* y1;
  int y1_cstride, y1_coff;
  // persistent patch kernel, frames whose last 32-px tile column holds <= 16 frame columns (the conv4 level's 240):
  // the odd (right-half) waves of those tiles hold no frame pixel and skip their MFMAs, and each XCD band walks its
  // last-column tiles after the others (with prot == 2's serpentine rounds the half-cost items pair up on the walkers
  // that hold the band's third round)
  int halfskip;
  // fp16 operands (VM_F16 input view and filter pack: the split-fp16 forward): the patch kernel's fp16 MFMA form
  int f16;
  // split-fp16 x3 output (vm_conv3x3_split3_nhwc; patch kernel f32-staged epilogue and the split-K reduction): y is
  // an fp16 view and each output value v (after bias / affine / act, in f32) is written as h = fp16(v), l =
  // fp16(v - h) into the slabs [l, h, h] at channel offsets 0, ysplit, 2 * ysplit; the fused pool likewise at
  // psplit.  ovf (device int, may be null) is set where |v| >= 65520 (the split would be invalid)
  int ysplit, psplit;
  int* ovf;
  // split-fp16 input stored as two slabs [l, h] of xalias channels (K = 3 * xalias: [l, h, h]): input channels
  // [2 * xalias, 3 * xalias) are read from [xalias, 2 * xalias) (src_chan), so h is stored once
  int xalias;
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [I, N)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// a pointer every lane holds the same value of, moved to SGPRs (buffer descriptors must be scalar)
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<P*>(((uint64_t)hi << 32) | lo);
}

// element offset of input channel c (relative to the view's channel 0) under the source split
__device__ __forceinline__ long src_chan(const ConvArgs& a, int c) {
  if (a.xalias > 0 && c >= 2 * a.xalias) c -= a.xalias;  // split-fp16 input: the third slab re-reads the second
  if (a.x_src_c <= 0) return c;
  const int s = c / a.x_src_c;
  return (long)s * a.x_src_stride + (c - s * a.x_src_c);
}

// LDS images are [row][RB bytes] with the 16-byte chunk index XOR-swizzled per row; both swizzles
// make the ds_read_b128 lane groups of a 16-row fragment read conflict-free from ANY starting row.
template <int RB>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (RB == 128) return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4);
}

// 2-bit chunk swizzle of 64-byte rows (the pair kernels' own patch images): like swz<64>, conflict-free for the
// ds_read_b128 fragment reads from any start row, and also for ds_write_b128 of 8 consecutive rows
__device__ __forceinline__ int swz2(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 3)) << 4); }

template <typename T>
__device__ __forceinline__ void mma16(const uint4& a, const uint4& b, f32x4& c);

template <>
__device__ __forceinline__ void mma16<uint16_t>(const uint4& a, const uint4& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                               0);
}

// fp16 operands (the split-fp16 x3 forward, vmatting/split3.py): 16-bit storage like bf16, so every bf16 data path
// (LDS-DMA, fragments, packing geometry) carries them unchanged; only the MFMA differs
template <>
__device__ __forceinline__ void mma16<f16_t>(const uint4& a, const uint4& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mma16<float>(const uint4& a, const uint4& b, f32x4& c) {
  // lane k-slot s = lane>>4 holds k = 4s..4s+3 of the 16-wide k-block; MFMA t consumes element t.
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
}

// split-fp16 x3 parts of 8 f32 values: h = fp16(v) (RNE), l = fp16(v - h) (the difference is exact in f32), as
// two 16-byte chunks; returns whether some |v| >= 65520 (h = inf: the split is invalid) or v is NaN
__device__ __forceinline__ bool split3h_chunk(const float* v, uint4& H, uint4& L) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  uint32_t wh[4], wl[4];
  bool ovf = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f2_t x = {v[2 * i], v[2 * i + 1]};
    const h2_t h = __builtin_convertvector(x, h2_t);
    wh[i] = __builtin_bit_cast(uint32_t, h);
    const f2_t r = {v[2 * i] - (float)h[0], v[2 * i + 1] - (float)h[1]};
    wl[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2_t));
    ovf |= !(fabsf(v[2 * i]) < 65520.f) || !(fabsf(v[2 * i + 1]) < 65520.f);
  }
  H = make_uint4(wh[0], wh[1], wh[2], wh[3]);
  L = make_uint4(wl[0], wl[1], wl[2], wl[3]);
  return ovf;
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD -> each XCD gets a contiguous tile range
__device__ __forceinline__ int xcd_tile(int b, int nwg) {
  const int q = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  return (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (b >> 3);
}

// bounds-checked buffer descriptors, rebased per block so 32-bit offsets cover any batch; a lane whose
// tap leaves the frame gets an out-of-range offset and the hardware returns 0 (SAME zero padding).
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x_rsrc(const ConvArgs& a, long xbase) {
  const T* Xb = reinterpret_cast<const T*>(a.x) + a.x_coff + xbase * (long)a.x_cstride;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Xb), 0, 0x7ffffff0, 0x00020000);
}
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w_rsrc(const ConvArgs& a, int n0) {
  const T* Wb = reinterpret_cast<const T*>(a.w) + (long)n0 * a.K_pad;
  const uint32_t bytes = (uint32_t)((long)(a.cout_pad - n0) * a.K_pad * (long)sizeof(T));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Wb), 0, bytes, 0x00020000);
}

constexpr int OOB = (int)0x80000000;
// the same for the issue-bound strip pair kernel: the bit pattern of -4.0f, an inline constant, so a select of it needs
// no v_bfrev to materialise 0x80000000 first (every descriptor here has num_records <= 0x7ffffff0).  Kept out of the
// MFMA-bound kernels, whose schedules measured 1 % slower with it (code placement, not the instruction count).
constexpr int OOB_INL = (int)0xC0800000;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(lds_ptr_t)(p);
}

// One 16-byte-per-lane LDS-DMA (buffer_load_dwordx4 ... offen lds) from inline asm.  Issued through asm on
// purpose: for a compiler-visible LDS-DMA, hipcc cannot prove the slot being read differs from the slots
// being filled and emits s_waitcnt vmcnt(0) before the next ds_read — draining every stage in flight.
// The asm is invisible to that bookkeeping; completion is counted by hand (wait_vm) before the barrier
// that publishes a slot.  M0 is compiler-reserved: set and restored inside the same statement.
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t rsrc, uint32_t lds_dst, int voffset) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voffset), "s"(lds_dst), "s"(rsrc)
      : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (immediate operand -> one case per value)
__device__ __forceinline__ void wait_vm(int n) {
#define VM_W(N) \
  case N:       \
    asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
    break;
  switch (n) {
    VM_W(0) VM_W(1) VM_W(2) VM_W(3) VM_W(4) VM_W(5) VM_W(6) VM_W(7) VM_W(8) VM_W(9) VM_W(10) VM_W(11) VM_W(12)
    VM_W(13) VM_W(14) VM_W(15) VM_W(16) VM_W(17) VM_W(18) VM_W(19) VM_W(20) VM_W(21) VM_W(22) VM_W(23) VM_W(24)
    VM_W(25) VM_W(26) VM_W(27) VM_W(28) VM_W(29) VM_W(30) VM_W(31) VM_W(32) VM_W(33) VM_W(34) VM_W(35) VM_W(36)
    VM_W(37) VM_W(38) VM_W(39) VM_W(40) VM_W(41) VM_W(42) VM_W(43) VM_W(44) VM_W(45) VM_W(46) VM_W(47) VM_W(48)
    VM_W(49) VM_W(50) VM_W(51) VM_W(52) VM_W(53) VM_W(54) VM_W(55) VM_W(56) VM_W(57) VM_W(58) VM_W(59) VM_W(60)
    VM_W(61) VM_W(62) VM_W(63)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef VM_W
}

// MFMA 16x16 output -> whole 16-byte channel chunks: lane (col, q) holds channels 4q..4q+3 of fragment pair member
// lo (channels 0..15 of a 32-channel group) and hi (16..31).  One v_permlane16_swap per dword trades the odd rows'
// lo with the even rows' hi, so even q holds channels 4q..4q+7 (chunk q/2) and odd q channels 16+4(q-1)..+7
// (chunk 2 + q/2) of the 32-channel group.
__device__ __forceinline__ uint4 chunk_pair(uint2 lo, uint2 hi) {
  const auto sx = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
  const auto sy = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
  return make_uint4(sx[0], sy[0], sx[1], sy[1]);
}

// name of the kernel the last conv call on this thread launched, spelled as rocprofv3 reports it (conv3x3.hip)
extern thread_local char g_last_kernel[128];

// vm_set_option "conv_prio": ConvArgs::prio for the 8-wave conv kernels (patch, persistent patch, row-stationary)
extern long g_conv_prio;
// launchers defined in conv_rows.hip (called from conv3x3.hip's dispatch)
bool rows_ok(const ConvArgs& a);
int launch_rows(ConvArgs& a, hipStream_t st, int cfg);
// launchers defined in conv_pair.hip
bool pair_strip_ok(const ConvArgs& a);
int launch_pair_strip(ConvArgs& a, long nimg, hipStream_t st);
extern long g_pair_strip_abl, g_pair_strip_pin;

}  // namespace vm
