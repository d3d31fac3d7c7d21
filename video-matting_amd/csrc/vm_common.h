// Shared helpers for the gfx950 kernels behind include/vmatting.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>

#include "vmatting.h"

namespace vm {

// per-thread error text for vm_last_error()
void set_error(const char* fmt, ...);

// tuning knobs of the training kernels (train.hip), reached through vm_set_option: 1 = handled, 0 = unknown key
int train_set_option(const char* key, long value);

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VM_EHIP, "%s: %s", what, hipGetErrorString(e));
  return VM_OK;
}

inline int elem_bytes(int dtype) { return dtype == VM_F32 ? 4 : (dtype == VM_BF16 || dtype == VM_F16) ? 2 : 1; }

// allow_f16: the conv input of the split-fp16 forward (vm_conv3x3_ex_nhwc / head_acc); every other op takes f32 / bf16
inline bool valid_tensor(const vm_tensor* t, bool allow_f16 = false) {
  return t && t->ptr && t->n > 0 && t->h > 0 && t->w > 0 && t->c > 0 && t->coff >= 0 &&
         t->coff + t->c <= t->cstride && (t->dtype == VM_F32 || t->dtype == VM_BF16 || (allow_f16 && t->dtype == VM_F16));
}

inline bool vec16_ok(const vm_tensor* t, int extra_elems_multiple = 1) {
  int ve = 16 / elem_bytes(t->dtype);
  return (reinterpret_cast<uintptr_t>(t->ptr) % 16 == 0) && (t->cstride % ve == 0) && (t->coff % ve == 0) &&
         (t->c % (ve * extra_elems_multiple) == 0);
}

// ---------------------------------------------------------------- device helpers
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// an IEEE fp16 element (VM_F16): 16-bit storage, a distinct type so templates pick the fp16 MFMA / conversions
struct f16_t {
  uint16_t v;
};

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);  // v_cvt_pk_bf16_f32 on gfx950: RNE, NaN stays NaN
  return __builtin_bit_cast(uint16_t, b);
}

// two floats -> packed bf16 pair (lo in bits 0..15): ONE v_cvt_pk_bf16_f32 with both operands, the same RNE rounding
// as f2bf.  Spelled as two f2bf calls, hipcc emits two conversions (second operand 0), a shift and an or.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bf16x2_bits(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

template <typename T>
__device__ __forceinline__ float ld_elem(const T* p);
template <>
__device__ __forceinline__ float ld_elem<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_elem<uint16_t>(const uint16_t* p) { return bf2f(*p); }

template <typename T>
__device__ __forceinline__ void st_elem(T* p, float v);
template <>
__device__ __forceinline__ void st_elem<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st_elem<uint16_t>(uint16_t* p, float v) { *p = f2bf(v); }
template <>
__device__ __forceinline__ void st_elem<f16_t>(f16_t* p, float v) {
  p->v = __builtin_bit_cast(uint16_t, static_cast<_Float16>(v));  // RNE
}

// 16-byte chunk <-> floats (4 f32 or 8 bf16)
template <typename T>
struct Chunk;
template <>
struct Chunk<float> {
  static constexpr int N = 4;
  __device__ static void unpack(uint4 u, float* f) {
    f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y);
    f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
  }
  __device__ static uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <>
struct Chunk<uint16_t> {
  static constexpr int N = 8;
  __device__ static void unpack(uint4 u, float* f) {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static uint4 pack(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = bf16x2_bits(f[2 * i], f[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == VM_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == VM_ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  return v;
}

// exact-ish sigmoid for the f32 parity path (expf, not the fast approximation)
__device__ __forceinline__ float sigmoid_precise(float v) {
  if (v >= 0.f) return 1.f / (1.f + expf(-v));
  float e = expf(v);
  return e / (1.f + e);
}

// pixel blocks of the BN partial-sum passes (elementwise.hip bn_partial_kernel, train.hip bn_bwd_partial): about
// g_bn_target blocks over all channel groups (vm_set_option "bn_blocks"), at least BN_NBLK_MIN per group, at most
// bn_max_blocks(C), which the workspaces are sized for.  1024 blocks (16 waves per CU) left the narrow full-resolution
// passes at ~2.5 TB/s; the partial sums are f64, so the block count only moves their rounding far below f32's.
constexpr int BN_NBLK_MIN = 1024, BN_TARGET_MAX = 8192;
extern long g_bn_target;
extern long g_bn_vec_fwd;  // elementwise.hip: the 8-channel forward BN forms (vm_set_option "bn_vec_fwd")
inline int bn_groups(int C) { return C > 32 ? (C + 63) / 64 : 1; }
inline int bn_max_blocks(int C) {
  const int t = BN_TARGET_MAX / bn_groups(C);
  return t > BN_NBLK_MIN ? t : BN_NBLK_MIN;
}
inline int bn_blocks(long M, int C) {
  long t = g_bn_target / bn_groups(C);
  if (t < BN_NBLK_MIN) t = BN_NBLK_MIN;
  if (t > bn_max_blocks(C)) t = bn_max_blocks(C);
  const long nb = M / 256 < t ? M / 256 : t;
  return nb < 1 ? 1 : (int)nb;
}

// channel c of k (<= 3) stacked channel-major [C][nblk] double tables (table j at part + j * nblk * C), summed by one
// 256-thread block: 4 partials' loads in flight per thread, then a wave shuffle tree and an LDS fold; the sums land
// in thread 0.  (r04: the tables were [nblk][C], so every load of the fold touched its own cache line — C * 8 bytes
// apart; channel-major they are one contiguous run per channel, the same values summed in the same order)
__device__ __forceinline__ void fold_columns(const double* part, int nblk, int C, int c, int k, double* out) {
  __shared__ double sh[3][4];
  double s[3] = {0.0, 0.0, 0.0};
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const long tab = (long)nblk * C;
  int b = t;
  for (; b + 3 * 256 < nblk; b += 4 * 256) {
    double v[3][4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) v[j][u] = j < k ? part[j * tab + (long)c * nblk + b + u * 256] : 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[j] += v[j][u];
  }
  for (; b < nblk; b += 256)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < k) s[j] += part[j * tab + (long)c * nblk + b];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    for (int o = 32; o > 0; o >>= 1) s[j] += __shfl_down(s[j], o);
    if (lane == 0) sh[j][wave] = s[j];
  }
  __syncthreads();
  if (t == 0)
#pragma unroll
    for (int j = 0; j < 3; ++j) out[j] = sh[j][0] + sh[j][1] + sh[j][2] + sh[j][3];
}

inline int grid_for(long work, int block, int max_blocks = 256 * 16) {
  long g = (work + block - 1) / block;
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

}  // namespace vm
