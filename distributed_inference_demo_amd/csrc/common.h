// common.h — shared types and device helpers for libbloomstage (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }  // RNE (v_cvt_pk_bf16_f32)

// Wave reductions without LDS: DPP butterflies inside each 16-lane row (xor 1, xor 2, rotate 4,
// rotate 8), then the four row results through v_readlane.  Every lane returns the total.
// (__shfl_xor lowers to ds_bpermute: six LDS round trips per reduction.)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  const int iv = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(iv, 0)) + __int_as_float(__builtin_amdgcn_readlane(iv, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(iv, 32)) + __int_as_float(__builtin_amdgcn_readlane(iv, 48)));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  const int iv = __float_as_int(v);
  return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(iv, 0)), __int_as_float(__builtin_amdgcn_readlane(iv, 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(iv, 32)), __int_as_float(__builtin_amdgcn_readlane(iv, 48))));
}

// Load 8 consecutive elements as fp32 (16 B for bf16, 32 B for fp32).
__device__ __forceinline__ void load8(const bf16* p, float* o) {
  u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = __uint_as_float(((uint32_t)v[j]) << 16);
}
__device__ __forceinline__ void load8(const float* p, float* o) {
  float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// bloom_gelu_forward (modeling_bloom.py:111-121), same evaluation order.
// BLOOM's tanh GELU (modeling_bloom.py bloom_gelu_forward): x/2 (1 + tanh u) = x sigmoid(2u) = x / (1 + e^-2u),
// one v_exp_f32 and one divide instead of tanhf's polynomial and branches (the prefill GEMM epilogue spent
// 8 us of a 27 us bloom-1b1 fc1 tile on tanhf); |difference| to the tanhf form is a few fp32 ulps of the
// result, under one bf16 rounding step of the stored activation.  u -> -inf: e^-2u = inf, x / inf = -0.
__device__ __forceinline__ float gelu_bloom(float x) {
  const float u = 0.79788456f * x * (1.0f + 0.044715f * x * x);
  return __fdividef(x, 1.0f + __expf(-2.0f * u));
}

// Weight loads (NT: non-temporal) and an 8-wide bf16 dot product on v_dot2c_f32_bf16.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int NT>
__device__ __forceinline__ bf16x8 wload(const bf16* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
  else return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[0], a[1]}, (bf16x2){b[0], b[1]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[2], a[3]}, (bf16x2){b[2], b[3]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[4], a[5]}, (bf16x2){b[4], b[5]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[6], a[7]}, (bf16x2){b[6], b[7]}, acc, false);
  return acc;
}

// Monotone float -> uint32 key (larger float => larger key).
__device__ __forceinline__ uint32_t f32_order_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// 8 consecutive elements kept in their storage type (bf16: 4 VGPRs) until used.
typedef float f32x8 __attribute__((ext_vector_type(8)));
template <typename T> struct Raw8;
template <> struct Raw8<bf16> { typedef u16x8 type; };
template <> struct Raw8<float> { typedef f32x8 type; };
__device__ __forceinline__ void raw_load(const bf16* p, u16x8& r) { r = *reinterpret_cast<const u16x8*>(p); }
__device__ __forceinline__ void raw_load(const float* p, f32x8& r) { r = *reinterpret_cast<const f32x8*>(p); }
__device__ __forceinline__ float raw_get(const u16x8& r, int j) { return __uint_as_float(((uint32_t)r[j]) << 16); }
__device__ __forceinline__ float raw_get(const f32x8& r, int j) { return r[j]; }
