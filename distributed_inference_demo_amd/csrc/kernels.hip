// kernels.hip — HIP kernels of one BLOOM pipeline stage, written for gfx950 (MI355X).
//
// Math restated from HF BLOOM (modeling_bloom.py; see oracle/bloom_oracle.c header for the
// line map) which is what the reference's ONNX sub-models execute (inference.cpp:207-215).
//
//  decode  (M = B*S <= 32):  gemv_mfma   — weight-streaming skinny GEMM on
//                            v_mfma_f32_16x16x32_bf16, split-K across the waves of a block,
//                            LDS reduction, fused epilogue.  HBM-bound.
//  prefill (M > 32):         gemm_mfma   — LDS double-buffered 16x16x32 bf16 MFMA tiles.
//  fp32 mode (parity):       gemm_f32    — exact-fp32 LDS-tiled GEMM.
//  attention: split-ctx decode (partial + combine) and a per-query online-softmax kernel
//  for S > 1; both causal + ALiBi over the contiguous per-stage KV cache.
#include <array>
#include <cstdio>
#include <cstring>
#include <vector>
#include "common.h"
#include "kernels.h"
#include "attn_merge.h"

// Buffer descriptor over a whole allocation for write-through / L2-coherent (aux = 16: sc1)
// accesses: the split partials other workgroups of the same launch read.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t attn_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0xFFFFFFFF, 0x00020000);
}

#include <algorithm>
#include <cstdlib>

// ------------------------------------------------------------------------------------
// Synthetic weights: device twin of oracle/gen.h (DESIGN.md "Synthetic weights").
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t d_sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ uint32_t d_lb32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t d_bits(uint64_t key, uint32_t i) {
  return d_lb32((uint32_t)key ^ d_lb32(i + (uint32_t)(key >> 32)));
}
__device__ __forceinline__ float d_gen_value(int kind, uint64_t key, uint64_t key2, uint32_t i) {
  if (kind == 0) {
    uint32_t h1 = d_bits(key, i), h2 = d_bits(key2, i);
    int s = 2 * (int)((h1 & 0xFFFFu) + (h1 >> 16) + (h2 & 0xFFFFu) + (h2 >> 16)) - 4 * 65535;
    return __fmul_rn((float)s, 0x1.1bc77ap-22f);
  }
  int s = 2 * (int)(d_bits(key, i) >> 8) - 16777215;
  if (kind == 1) return __fmul_rn((float)s, 0x1.47ae14p-30f);
  float t = __fmul_rn((float)s, 0x1.99999ap-28f);
  // gamma = 1 + s*c must round twice (like the C and numpy twins): the empty asm makes t
  // opaque so the add cannot be fused into a v_fma_f32.
  asm volatile("" : "+v"(t));
  return kind == 2 ? __fadd_rn(1.0f, t) : t;
}

template <typename T>
__global__ void gen_fill_kernel(T* dst, uint64_t n, uint64_t key, uint64_t key2, int kind, uint64_t off) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = from_f32<T>(d_gen_value(kind, key, key2, (uint32_t)(i + off)));
}

template <typename T>
__global__ void convert_kernel(T* dst, const float* src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = from_f32<T>(src[i]);
}

static uint64_t h_sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void launch_gen_fill(void* dst, int is_bf16, uint64_t n, uint64_t key, int kind, hipStream_t s, uint64_t off) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return;
  if (is_bf16)
    gen_fill_kernel<bf16><<<(unsigned)blocks, 256, 0, s>>>((bf16*)dst, n, key, h_sm64(key), kind, off);
  else
    gen_fill_kernel<float><<<(unsigned)blocks, 256, 0, s>>>((float*)dst, n, key, h_sm64(key), kind, off);
}

void launch_convert_f32(void* dst, int is_bf16, const float* src, uint64_t n, hipStream_t s) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return;
  if (is_bf16) convert_kernel<bf16><<<(unsigned)blocks, 256, 0, s>>>((bf16*)dst, src, n);
  else convert_kernel<float><<<(unsigned)blocks, 256, 0, s>>>((float*)dst, src, n);
}

// ------------------------------------------------------------------------------------
// LayerNorm (nn.LayerNorm: biased variance, eps inside the sqrt), one row per block.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float block_sum_256(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

template <typename TI, typename T, typename TO>
__global__ __launch_bounds__(256) void layernorm_kernel(const TI* __restrict__ x, const int* __restrict__ ids,
                                                         int row_stride, int row_offset,
                                                         const T* __restrict__ g, const T* __restrict__ b,
                                                         TO* __restrict__ out, int K, float eps) {
  __shared__ float sh[4];
  const int m = blockIdx.x;
  const TI* xr = ids ? x + (size_t)ids[m] * K : x + ((size_t)m * row_stride + row_offset) * K;
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) s += to_f32(xr[k]);
  const float mean = block_sum_256(s, sh) / (float)K;
  float v = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) { float d = to_f32(xr[k]) - mean; v += d * d; }
  const float var = block_sum_256(v, sh) / (float)K;
  const float rstd = 1.0f / sqrtf(var + eps);
  TO* o = out + (size_t)m * K;
  for (int k = threadIdx.x; k < K; k += 256)
    o[k] = from_f32<TO>((to_f32(xr[k]) - mean) * rstd * to_f32(g[k]) + to_f32(b[k]));
}

void launch_layernorm(int is_bf16, const void* x, const int* ids, int row_stride, int row_offset,
                      const void* gamma, const void* beta, void* out, int out_f32, int M, int K,
                      float eps, hipStream_t s) {
  if (M <= 0) return;
  if (is_bf16) {
    if (ids) {
      layernorm_kernel<bf16, bf16, float><<<M, 256, 0, s>>>((const bf16*)x, ids, 0, 0, (const bf16*)gamma,
                                                            (const bf16*)beta, (float*)out, K, eps);
    } else if (out_f32) {
      layernorm_kernel<float, bf16, float><<<M, 256, 0, s>>>((const float*)x, nullptr, row_stride, row_offset,
                                                             (const bf16*)gamma, (const bf16*)beta, (float*)out, K, eps);
    } else {
      layernorm_kernel<float, bf16, bf16><<<M, 256, 0, s>>>((const float*)x, nullptr, row_stride, row_offset,
                                                            (const bf16*)gamma, (const bf16*)beta, (bf16*)out, K, eps);
    }
  } else {
    layernorm_kernel<float, float, float><<<M, 256, 0, s>>>((const float*)x, ids, ids ? 0 : row_stride,
                                                            ids ? 0 : row_offset, (const float*)gamma,
                                                            (const float*)beta, (float*)out, K, eps);
  }
}

// ------------------------------------------------------------------------------------
// Fused epilogues.
// ------------------------------------------------------------------------------------
// 16 consecutive lanes (same lane>>4) hold the 16 columns of one output row: reduce the
// (value, column) argmax over them and let the column-0 lane store the tile's key.
__device__ __forceinline__ void argmax_tile16(const Epi& e, int m, int n, float v, bool valid, int ntiles) {
  const uint32_t col = (uint32_t)(n + e.col_offset);
  unsigned long long key =
      valid ? (((unsigned long long)f32_order_key(v) << 32) | (e.key_hi_index ? col : 0xFFFFFFFFu - col)) : 0ull;
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) {
    unsigned long long other = __shfl_xor(key, o, 64);
    key = other > key ? other : key;
  }
  if (valid && (n & 15) == 0) e.keys[(size_t)m * ntiles + (n >> 4)] = key;
  if (valid && e.logits) e.logits[(size_t)m * e.ldo + n] = v;
}

template <typename T, int KIND>
__device__ __forceinline__ void epi_store(const Epi& e, int m, int n, float v) {
  if (e.col_scale) v *= e.col_scale[n];
  if constexpr (KIND == EPI_QKV) {
    v += to_f32(((const T*)e.bias)[n]);
    const int three = 3 * e.head_dim;
    const int head = n / three, r = n - head * three, which = r / e.head_dim, d = r - which * e.head_dim;
    if (which == 0) {
      ((T*)e.q_out)[(size_t)m * e.hidden + head * e.head_dim + d] = from_f32<T>(v);
    } else {
      const int b = m / e.seq, t = m - b * e.seq;
      const int past = e.past_dev ? e.past_dev[b] : e.past;
      const size_t idx = (((size_t)(e.slot + b) * e.n_head + head) * e.max_ctx + past + t) * e.head_dim + d;
      T* c = (T*)(which == 1 ? e.k_cache : e.v_cache);
      c[idx] = from_f32<T>(v);
    }
  } else if constexpr (KIND == EPI_RESID) {
    const size_t i = (size_t)m * e.ldo + n;
    e.out_f32[i] = (v + to_f32(((const T*)e.bias)[n])) + e.resid[i];
  } else if constexpr (KIND == EPI_GELU) {
    ((T*)e.out_act)[(size_t)m * e.ldo + n] = from_f32<T>(gelu_bloom(v + to_f32(((const T*)e.bias)[n])));
  }
}

// Epilogue operands that do not depend on the GEMV result (bias, residual, past_len): a GEMV whose
// output lane is known up front loads them at kernel start, so the epilogue is not one more memory
// round trip after the reduction (decode GEMVs are latency-bound; each round trip is ~1 us).
struct EpiPre {
  uint32_t bias_bits;  // raw storage bits of bias[n] (bf16: low 16 bits), converted where used
  float resid;
  int past;
};

template <typename T>
__device__ __forceinline__ float bias_value(uint32_t bits) {
  if constexpr (sizeof(T) == 2) return __uint_as_float(bits << 16);
  else return __uint_as_float(bits);
}

// The loads go out unconditionally (lanes without an output read index 0) and stay raw until the
// epilogue: a value converted here, or loaded under an exec-masked branch, makes the compiler wait
// for it at once -- a whole HBM round trip before the weight stream is even issued.
template <typename T>
__device__ __forceinline__ EpiPre epi_prefetch(const Epi& e, int m, int n, bool valid) {
  EpiPre p{0u, 0.f, 0};
  if (e.kind == EPI_ARGMAX) return p;  // uniform (kernel argument)
  const int nn = valid ? n : 0, mm = valid ? m : 0;
  if constexpr (sizeof(T) == 2) p.bias_bits = ((const unsigned short*)e.bias)[nn];
  else p.bias_bits = ((const uint32_t*)e.bias)[nn];
  if (e.kind == EPI_RESID) p.resid = e.resid[(size_t)mm * e.ldo + nn];
  if (e.kind == EPI_QKV) p.past = e.past_dev ? e.past_dev[mm / e.seq] : e.past;
  return p;
}

// epi_store with the operands from epi_prefetch (same arithmetic, same roundings).
template <typename T, int KIND>
__device__ __forceinline__ void epi_store_pre(const Epi& e, int m, int n, float v, const EpiPre& p) {
  if (e.col_scale) v *= e.col_scale[n];
  const float bias = bias_value<T>(p.bias_bits);
  if constexpr (KIND == EPI_QKV) {
    v += bias;
    const int three = 3 * e.head_dim;
    const int head = n / three, r = n - head * three, which = r / e.head_dim, d = r - which * e.head_dim;
    if (which == 0) {
      ((T*)e.q_out)[(size_t)m * e.hidden + head * e.head_dim + d] = from_f32<T>(v);
    } else {
      const int b = m / e.seq, t = m - b * e.seq;
      const size_t idx = (((size_t)(e.slot + b) * e.n_head + head) * e.max_ctx + p.past + t) * e.head_dim + d;
      T* c = (T*)(which == 1 ? e.k_cache : e.v_cache);
      c[idx] = from_f32<T>(v);
    }
  } else if constexpr (KIND == EPI_RESID) {
    e.out_f32[(size_t)m * e.ldo + n] = (v + bias) + p.resid;
  } else if constexpr (KIND == EPI_GELU) {
    ((T*)e.out_act)[(size_t)m * e.ldo + n] = from_f32<T>(gelu_bloom(v + bias));
  }
}

// Apply the epilogue of compile-time kind K to one element (argmax needs all 64 lanes).
template <typename T, int K>
__device__ __forceinline__ void epi_apply(const Epi& ep, int m, int n, float v, bool valid, int ntiles) {
  if constexpr (K == EPI_ARGMAX) argmax_tile16(ep, m, n, v, valid, ntiles);
  else if (valid) epi_store<T, K>(ep, m, n, v);
}

template <int V> struct EpiKindC { static constexpr int value = V; };

// Call f(EpiKindC<kind>) so the epilogue kind is a compile-time constant inside f: each kind's
// loop nest then unrolls on its own (a runtime switch inside an unrolled accumulator loop
// stops the unrolling and sends the accumulators to scratch).
template <typename F>
__device__ __forceinline__ void epi_dispatch(int kind, F&& f) {
  switch (kind) {
    case EPI_QKV: f(EpiKindC<EPI_QKV>{}); break;
    case EPI_RESID: f(EpiKindC<EPI_RESID>{}); break;
    case EPI_GELU: f(EpiKindC<EPI_GELU>{}); break;
    default: f(EpiKindC<EPI_ARGMAX>{}); break;
  }
}

// ------------------------------------------------------------------------------------
// gemv_mfma: out[m][n] for M <= 16*MT rows.  Block = one 16-column tile of W, WAVES waves
// split K; each wave streams its K range of the 16 weight rows straight to VGPRs (16 B per
// lane, U k-steps in flight) and runs one v_mfma_f32_16x16x32_bf16 per k-step and m-tile
// with A = W tile (rows = n), B = X^T (cols = m).  Partial tiles meet in LDS.
// ------------------------------------------------------------------------------------
// LN variant (LN = true, M <= 8): X is the fp32 residual stream; the block computes the
// LayerNorm statistics of its M rows (two passes, L2-resident) while its first U weight
// loads are in flight, writes the normalised bf16 rows to LDS, and reads B fragments there.
struct LnArgs {
  const float* x;     // fp32 rows; source row of m = m * row_stride + row_offset
  int row_stride, row_offset;
  const bf16* gamma;
  const bf16* beta;
  float eps;
  // X_EMB (gemv_rows_kernel, the first stage's layer 0): row m is word_embeddings[ids[m]] normalised by
  // word_embeddings_layernorm (emb_g, emb_b) in fp32 -- the residual stream, stored by block 0 to x_out --
  // and then by (gamma, beta) as X_LN.  `x` is unused.
  const int* ids;
  const bf16* wemb;
  const bf16* emb_g;
  const bf16* emb_b;
  float* x_out;
};

// NT: non-temporal weight loads; PF: prefetch the next U weight steps before this step's MFMAs.
template <int WAVES, int MT, int U, bool LN, int NT = 1, int PF = 1>
__global__ __launch_bounds__(WAVES * 64) void gemv_mfma_kernel(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                                               LnArgs ln, int M, int N, int K, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float (*red)[MT * 16][17] = reinterpret_cast<float (*)[MT * 16][17]>(smem);
  bf16* xs = reinterpret_cast<bf16*>(smem + sizeof(float) * WAVES * MT * 16 * 17);  // LN: [M][K]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const bf16* wp = W + (size_t)min(n0 + r, N - 1) * K + g * 8;
  const int ksteps = K >> 5;
  const int per = (ksteps + WAVES - 1) / WAVES;
  const int s0 = w * per, s1 = min(ksteps, s0 + per);
  auto wload = [&](int ss) -> bf16x8 {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(wp + (size_t)ss * 32);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
  };
  bf16x8 a[U];
  if (PF && s0 < s1) {
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = wload(min(s0 + u, s1 - 1));
  }
  const bf16* xp[MT];
  if constexpr (LN) {
    // ---- LayerNorm prologue (nn.LayerNorm: biased variance, eps inside the sqrt)
    float* st = &red[0][0][0];  // reuse: [2][8] stats + [WAVES][8] partials
    float part[8];
    const int nthr = WAVES * 64;
#pragma unroll
    for (int m = 0; m < 8; m++) part[m] = 0.f;
#pragma unroll
    for (int m = 0; m < 8; m++) {
      if (m < M) {
        const float* xr = ln.x + ((size_t)m * ln.row_stride + ln.row_offset) * K;
        float acc = 0.f;
        for (int k = threadIdx.x * 4; k < K; k += nthr * 4) {
          const float4 v = *reinterpret_cast<const float4*>(xr + k);
          acc += (v.x + v.y) + (v.z + v.w);
        }
        part[m] = wave_sum(acc);
      }
    }
    float* wp_part = st + 16;
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < 8; m++)
        if (m < M) wp_part[w * 8 + m] = part[m];
    }
    __syncthreads();
    if (threadIdx.x < M) {
      float t = 0.f;
      for (int ww = 0; ww < WAVES; ww++) t += wp_part[ww * 8 + threadIdx.x];
      st[threadIdx.x] = t / (float)K;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; m++) {
      if (m < M) {
        const float* xr = ln.x + ((size_t)m * ln.row_stride + ln.row_offset) * K;
        const float mean = st[m];
        float acc = 0.f;
        for (int k = threadIdx.x * 4; k < K; k += nthr * 4) {
          const float4 v = *reinterpret_cast<const float4*>(xr + k);
          const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
          acc += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
        part[m] = wave_sum(acc);
      }
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < 8; m++)
        if (m < M) wp_part[w * 8 + m] = part[m];
    }
    __syncthreads();
    if (threadIdx.x < M) {
      float t = 0.f;
      for (int ww = 0; ww < WAVES; ww++) t += wp_part[ww * 8 + threadIdx.x];
      st[8 + threadIdx.x] = 1.0f / sqrtf(t / (float)K + ln.eps);
    }
    __syncthreads();
    for (int m = 0; m < M; m++) {
      const float* xr = ln.x + ((size_t)m * ln.row_stride + ln.row_offset) * K;
      const float mean = st[m], rstd = st[8 + m];
      for (int k = threadIdx.x * 8; k < K; k += nthr * 8) {
        float xv[8], gv[8], bv[8];
        load8(xr + k, xv);
        load8(ln.gamma + k, gv);
        load8(ln.beta + k, bv);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = (bf16)((xv[j] - mean) * rstd * gv[j] + bv[j]);
        *reinterpret_cast<bf16x8*>(xs + (size_t)m * K + k) = o;
      }
    }
    __syncthreads();
#pragma unroll
    for (int mt = 0; mt < MT; mt++) xp[mt] = xs + (size_t)min(mt * 16 + r, M - 1) * K + g * 8;
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; mt++) xp[mt] = X + (size_t)min(mt * 16 + r, M - 1) * K + g * 8;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // U k-steps per iteration, always fully unrolled: the steps past s1 re-load step s1-1
  // (an L1/L2 hit) and contribute a zeroed B fragment, so a short K range still keeps U
  // weight loads in flight instead of falling into a one-load-at-a-time remainder loop.
  // The next iteration's weights are loaded before this iteration's MFMAs.
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  for (int s = s0; s < s1; s += U) {
    if constexpr (!PF) {
#pragma unroll
      for (int u = 0; u < U; u++) a[u] = wload(min(s + u, s1 - 1));
    }
    bf16x8 b[MT][U];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int ss = min(s + u, s1 - 1);
        b[mt][u] = *reinterpret_cast<const bf16x8*>(xp[mt] + (size_t)ss * 32);
      }
    bf16x8 an[U];
    const bool more = PF && s + U < s1;
    if (more) {
#pragma unroll
      for (int u = 0; u < U; u++) an[u] = wload(min(s + U + u, s1 - 1));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const bool live = s + u < s1;
#pragma unroll
      for (int mt = 0; mt < MT; mt++)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], live ? b[mt][u] : zero8, acc[mt], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < U; u++) a[u] = an[u];
    }
  }
  if constexpr (LN) __syncthreads();  // red aliases the stats scratch
  // D[row = 4g+i (n)][col = r (m)]
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int i = 0; i < 4; i++) red[w][mt * 16 + r][4 * g + i] = acc[mt][i];
  __syncthreads();
  const int ntiles = (N + 15) >> 4;
  epi_dispatch(ep.kind, [&](auto kc) {
    constexpr int EK = decltype(kc)::value;
    for (int t = threadIdx.x; t < MT * 256; t += WAVES * 64) {
      const int ml = t >> 4, nl = t & 15;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ww++) v += red[ww][ml][nl];
      const int n = n0 + nl;
      epi_apply<bf16, EK>(ep, ml, n, v, ml < M && n < N, ntiles);
    }
  });
}

// ------------------------------------------------------------------------------------
// gemv_rows: decode GEMV for M <= MM <= 4.  Each wave owns R consecutive weight rows and streams
// them whole: every load instruction reads 1 KB contiguous (64 lanes x 16 B of one row), U
// 512-column chunks per row in flight.  Dot products on v_dot2c_f32_bf16 against x (bf16, from
// LDS for the LN variant, which normalises the rows there, else from global/L1).  Partial sums
// per lane are reduced across the wave at the end.  Small blocks (4 waves) and one wave per
// 1-4 rows give every CU several blocks, so no wave-quantisation tail on N = h GEMVs.
// ------------------------------------------------------------------------------------

// LayerNorm of M <= MM <= 4 rows (K <= 4096) into LDS as bf16, 256 threads, nn.LayerNorm
// semantics.  Each thread keeps its <= 16 values per row in registers: one global pass, ONE block
// reduction of the shifted sums (x - c, (x - c)^2 with c = the row's first element, which keeps
// the one-pass variance free of cancellation when |mean| >> std), normalise from registers.  Split
// in two so a kernel can put its own loads (the weight stream) between the row loads and the math.
template <int MM>
__device__ __forceinline__ void ln_rows_load(const LnArgs& ln, int M, int K, float4 (&xv)[MM][4], float (&c)[MM],
                                             uint2 (&gb)[4][2]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {  // gamma/beta with the rows: no round trip after the reductions
    const int k = threadIdx.x * 4 + i * 1024;
    gb[i][0] = k < K ? *reinterpret_cast<const uint2*>(ln.gamma + k) : make_uint2(0u, 0u);
    gb[i][1] = k < K ? *reinterpret_cast<const uint2*>(ln.beta + k) : make_uint2(0u, 0u);
  }
#pragma unroll
  for (int m = 0; m < MM; m++) {
    const float* xr = ln.x + ((size_t)min(m, M - 1) * ln.row_stride + ln.row_offset) * K;
    c[m] = xr[0];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int k = threadIdx.x * 4 + i * 1024;
      xv[m][i] = k < K ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// Threads >= 256 of a wider block take no part (their loads were never issued) but pass the barriers.
template <int MM>
__device__ __forceinline__ void ln_rows_finish(const LnArgs& ln, int M, int K, float4 (&xv)[MM][4],
                                               const float (&c)[MM], const uint2 (&gb)[4][2], bf16* xs,
                                               float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool active = threadIdx.x < 256;
  float s1[MM], s2[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) {
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (threadIdx.x * 4 + i * 1024 < K) {
        const float d0 = xv[m][i].x - c[m], d1 = xv[m][i].y - c[m], d2 = xv[m][i].z - c[m], d3 = xv[m][i].w - c[m];
        a1 += (d0 + d1) + (d2 + d3);
        a2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
    s1[m] = wave_sum(a1);
    s2[m] = wave_sum(a2);
  }
  if (lane == 0 && active) {
#pragma unroll
    for (int m = 0; m < MM; m++) {
      scratch[w * 8 + m] = s1[m];
      scratch[32 + w * 8 + m] = s2[m];
    }
  }
  __syncthreads();
  float mean[MM], rstd[MM];
  const float invk = 1.0f / (float)K;
#pragma unroll
  for (int m = 0; m < MM; m++) {
    const float t1 = ((scratch[m] + scratch[8 + m]) + (scratch[16 + m] + scratch[24 + m])) * invk;
    const float t2 = ((scratch[32 + m] + scratch[40 + m]) + (scratch[48 + m] + scratch[56 + m])) * invk;
    mean[m] = c[m] + t1;
    rstd[m] = 1.0f / sqrtf(fmaxf(t2 - t1 * t1, 0.f) + ln.eps);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int k = threadIdx.x * 4 + i * 1024;
    if (k < K && active) {
      const uint2 graw = gb[i][0], braw = gb[i][1];
      const float g[4] = {__uint_as_float(graw.x << 16), __uint_as_float(graw.x & 0xFFFF0000u),
                          __uint_as_float(graw.y << 16), __uint_as_float(graw.y & 0xFFFF0000u)};
      const float bb[4] = {__uint_as_float(braw.x << 16), __uint_as_float(braw.x & 0xFFFF0000u),
                           __uint_as_float(braw.y << 16), __uint_as_float(braw.y & 0xFFFF0000u)};
#pragma unroll
      for (int m = 0; m < MM; m++) {
        if (m < M) {
          const float v[4] = {xv[m][i].x, xv[m][i].y, xv[m][i].z, xv[m][i].w};
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; j++) o[j] = (bf16)((v[j] - mean[m]) * rstd[m] * g[j] + bb[j]);
          *reinterpret_cast<bf16x4*>(xs + (size_t)m * K + k) = o;
        }
      }
    }
  }
  __syncthreads();
}

// LayerNorm of M fp32 rows (K <= 4096, K % 4 == 0) -> bf16 with WPR waves per row (a 64 * WPR-thread block): the row
// in registers (NV float4 per lane; lane l of wave w holds float4 groups i * 64 * WPR + w * 64 + l), the shifted-sum
// statistics of ln_rows_finish by DPP wave reductions, and for WPR > 1 one LDS exchange of the WPR wave sums (added in
// wave order).  Round 4 went from a 256-thread block per row (two block barriers) to one wave per row; round 6
// measured one wave per row latency-bound at wide rows (tools/ln_bench.hip, profiles/r06_ln_rows_ab.txt: bloom-7b1
// K = 4096 4.9-5.1 us, 4 waves per row 2.8-3.0 us; 3b 3.9 -> 2.7; 1b1 2.8-3.0 -> 2.6-2.7), so rows wider than 1024
// take 4 waves.
template <int NV, int WPR>
__global__ __launch_bounds__(64 * WPR) void ln_rows_wave_kernel(LnArgs ln, int K, bf16* __restrict__ out) {
  __shared__ float sh[2 * WPR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* xr = ln.x + (size_t)blockIdx.x * ln.row_stride * K + (size_t)ln.row_offset * K;
  float4 xv[NV];
  uint2 gr[NV], br[NV];
  const float c = xr[0];
#pragma unroll
  for (int i = 0; i < NV; i++) {
    const int k = (i * 64 * WPR + w * 64 + lane) * 4;
    xv[i] = k < K ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    gr[i] = k < K ? *reinterpret_cast<const uint2*>(ln.gamma + k) : make_uint2(0u, 0u);
    br[i] = k < K ? *reinterpret_cast<const uint2*>(ln.beta + k) : make_uint2(0u, 0u);
  }
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    if ((i * 64 * WPR + w * 64 + lane) * 4 < K) {
      const float d0 = xv[i].x - c, d1 = xv[i].y - c, d2 = xv[i].z - c, d3 = xv[i].w - c;
      a1 += (d0 + d1) + (d2 + d3);
      a2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if constexpr (WPR > 1) {
    if (lane == 0) { sh[w] = a1; sh[WPR + w] = a2; }
    __syncthreads();
    a1 = sh[0]; a2 = sh[WPR];
#pragma unroll
    for (int j = 1; j < WPR; j++) { a1 += sh[j]; a2 += sh[WPR + j]; }
  }
  const float invk = 1.0f / (float)K;
  const float t1 = a1 * invk, t2 = a2 * invk;
  const float mean = c + t1, rstd = 1.0f / sqrtf(fmaxf(t2 - t1 * t1, 0.f) + ln.eps);
  bf16* orow = out + (size_t)blockIdx.x * K;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    const int k = (i * 64 * WPR + w * 64 + lane) * 4;
    if (k < K) {
      float4 g, b;
      bf16x4_to_f32(gr[i], g);
      bf16x4_to_f32(br[i], b);
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 o;
      o[0] = (bf16)((xv[i].x - mean) * rstd * g.x + b.x);
      o[1] = (bf16)((xv[i].y - mean) * rstd * g.y + b.y);
      o[2] = (bf16)((xv[i].z - mean) * rstd * g.z + b.z);
      o[3] = (bf16)((xv[i].w - mean) * rstd * g.w + b.w);
      *reinterpret_cast<bf16x4*>(orow + k) = o;
    }
  }
}

// K <= 4096, K % 4 == 0: one wave per row up to K = 1024 (NV = K / 256 float4 per lane), 4 waves per row above.
static void launch_ln_rows_wave(const LnArgs& ln, int M, int K, bf16* out, hipStream_t s) {
  if (K <= 1024) {
    ln_rows_wave_kernel<4, 1><<<M, 64, 0, s>>>(ln, K, out);
    return;
  }
  const int nv = (K + 1023) / 1024;
  if (nv <= 2) ln_rows_wave_kernel<2, 4><<<M, 256, 0, s>>>(ln, K, out);
  else ln_rows_wave_kernel<4, 4><<<M, 256, 0, s>>>(ln, K, out);
}

// Diagnostic builds only (tools/gemv_timeline.hip defines BS_STAMPS): wave 0 of every block records
// s_memrealtime (100 MHz, chip-wide) at kernel entry, after the prologue, after the K loop and after the
// epilogue.  The product library never defines it.
#ifdef BS_STAMPS
__device__ unsigned long long g_stamps[65536 * 4];
#define BS_STAMP(i) do { if (threadIdx.x == 0) g_stamps[blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BS_STAMP(i) do {} while (0)
#endif

// Activation prologue of gemv_rows_kernel: X read as given, LayerNorm of fp32 rows, or the merge
// of split-attention partials (attn_merge.h); the last two stage bf16 rows in LDS.
enum XMode : int { X_PLAIN = 0, X_LN = 1, X_PARTS = 2, X_EMB = 3 };
constexpr int kPartsPre = 2;  // 4-column groups per thread whose partial loads go out before the weights

// Two-pass LayerNorm statistics (mean, then centred squares) of M <= MM rows held by the first 256
// threads (thread t: columns t*4 + i*1024, i < 4, below K); every thread of the block returns them.
template <int MM>
__device__ __forceinline__ void ln_stats_256(const float4 (&v)[MM][4], int K, float eps, float* scratch,
                                             float (&mean)[MM], float (&rstd)[MM]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool active = threadIdx.x < 256;
  const float invk = 1.0f / (float)K;
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
#pragma unroll
    for (int m = 0; m < MM; m++) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (active && (int)threadIdx.x * 4 + i * 1024 < K) {
          if (pass == 0) a += (v[m][i].x + v[m][i].y) + (v[m][i].z + v[m][i].w);
          else {
            const float d0 = v[m][i].x - mean[m], d1 = v[m][i].y - mean[m], d2 = v[m][i].z - mean[m], d3 = v[m][i].w - mean[m];
            a += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
          }
        }
      }
      a = wave_sum(a);
      if (lane == 0 && active) scratch[pass * 32 + w * 8 + m] = a;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MM; m++) {
      const float t = ((scratch[pass * 32 + m] + scratch[pass * 32 + 8 + m]) +
                       (scratch[pass * 32 + 16 + m] + scratch[pass * 32 + 24 + m])) * invk;
      if (pass == 0) mean[m] = t;
      else rstd[m] = 1.0f / sqrtf(t + eps);
    }
  }
  __syncthreads();  // scratch is reused by the caller
}

__device__ __forceinline__ void bf16x4_to_f32(const uint2 raw, float4& o) {
  o = make_float4(__uint_as_float(raw.x << 16), __uint_as_float(raw.x & 0xFFFF0000u),
                  __uint_as_float(raw.y << 16), __uint_as_float(raw.y & 0xFFFF0000u));
}

// X_EMB, part 1 (before the weight stream is issued): the ids and both LayerNorms' gamma / beta.
template <int MM>
__device__ __forceinline__ void emb_rows_prefetch(const LnArgs& ln, int M, int K, int (&id)[MM], uint2 (&egb)[4][2],
                                                  uint2 (&gb)[4][2]) {
#pragma unroll
  for (int m = 0; m < MM; m++) id[m] = ln.ids[min(m, M - 1)];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int k = min((int)threadIdx.x * 4 + i * 1024, K - 4);
    egb[i][0] = *reinterpret_cast<const uint2*>(ln.emb_g + k);
    egb[i][1] = *reinterpret_cast<const uint2*>(ln.emb_b + k);
    gb[i][0] = *reinterpret_cast<const uint2*>(ln.gamma + k);
    gb[i][1] = *reinterpret_cast<const uint2*>(ln.beta + k);
  }
}

// Part 2: gather the embedding rows, word_embeddings_layernorm (fp32; block 0 stores it as the residual
// stream), then the layer's LN_in to bf16 rows in LDS.  The row loads are issued behind the weight stream
// (they need the ids), so this part waits for the block's first weight chunks too.
template <int MM>
__device__ __forceinline__ void emb_rows_finish(const LnArgs& ln, int M, int K, const int (&id)[MM],
                                                const uint2 (&egb)[4][2], const uint2 (&gb)[4][2], bf16* xs,
                                                float* scratch) {
  float4 v[MM][4];
#pragma unroll
  for (int m = 0; m < MM; m++) {
    const bf16* row = ln.wemb + (size_t)id[m] * K;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int k = min((int)threadIdx.x * 4 + i * 1024, K - 4);
      bf16x4_to_f32(*reinterpret_cast<const uint2*>(row + k), v[m][i]);
    }
  }
  float mean[MM], rstd[MM];
  ln_stats_256<MM>(v, K, ln.eps, scratch, mean, rstd);
  const bool active = threadIdx.x < 256;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    float4 g, b;
    bf16x4_to_f32(egb[i][0], g);
    bf16x4_to_f32(egb[i][1], b);
    const int k = (int)threadIdx.x * 4 + i * 1024;
#pragma unroll
    for (int m = 0; m < MM; m++) {
      v[m][i].x = (v[m][i].x - mean[m]) * rstd[m] * g.x + b.x;
      v[m][i].y = (v[m][i].y - mean[m]) * rstd[m] * g.y + b.y;
      v[m][i].z = (v[m][i].z - mean[m]) * rstd[m] * g.z + b.z;
      v[m][i].w = (v[m][i].w - mean[m]) * rstd[m] * g.w + b.w;
      if (blockIdx.x == 0 && active && k < K && m < M) *reinterpret_cast<float4*>(ln.x_out + (size_t)m * K + k) = v[m][i];
    }
  }
  ln_stats_256<MM>(v, K, ln.eps, scratch, mean, rstd);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int k = (int)threadIdx.x * 4 + i * 1024;
    if (active && k < K) {
      float4 g, b;
      bf16x4_to_f32(gb[i][0], g);
      bf16x4_to_f32(gb[i][1], b);
#pragma unroll
      for (int m = 0; m < MM; m++) {
        if (m < M) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 o;
          o[0] = (bf16)((v[m][i].x - mean[m]) * rstd[m] * g.x + b.x);
          o[1] = (bf16)((v[m][i].y - mean[m]) * rstd[m] * g.y + b.y);
          o[2] = (bf16)((v[m][i].z - mean[m]) * rstd[m] * g.z + b.z);
          o[3] = (bf16)((v[m][i].w - mean[m]) * rstd[m] * g.w + b.w);
          *reinterpret_cast<bf16x4*>(xs + (size_t)m * K + k) = o;
        }
      }
    }
  }
  __syncthreads();
}

// FL: probe flags for tools/gemv_probe.hip (0 in the product): 1 = temporal (not non-temporal) weight loads,
// 2 = no activation loads (x = 1), 4 = no epilogue (a store that never fires keeps the math).
// Block = blockDim.x / 64 waves (1..16): the dispatch sizes blocks so the grid is ~one block per CU
// and every CU streams the same number of weight bytes (gemv_rows_dispatch).
// The block body, also used by tools/attn_dense_fused.hip's one-launch attention + dense experiment (measured slower,
// not in the library; the library always passes wait = nullptr): block `bid`.  wait != nullptr (X_PARTS there): the
// split-attention partials come from the SAME launch -- the weight stream is issued first, then one lane polls *wait
// (sc1 loads) until it reaches `target` (bounded: ~0.2 s, then wait[2] = 1 records the timeout), the block meets
// at a barrier, and every partial load is an sc1 load (MI355X_MICROARCH.md "Valid forms" row 1).
// SYNC (compile time): only the tool instantiates the in-launch wait; in the library it is compiled out.
template <int R, int MM, int U, int XM, int FL = 0, bool SYNC = false>
__device__ __forceinline__ void gemv_rows_block(const bf16* __restrict__ W, const bf16* __restrict__ X, const LnArgs& ln,
                                                const AttnParts& pa, int M, int N, int K, const Epi& ep, int bid,
                                                char* smem, unsigned* wait, unsigned target) {
  if constexpr (!SYNC) wait = nullptr;  // every poll / sc1 path below folds away
  constexpr bool LN = XM == X_LN;
  BS_STAMP(0);
  float* scratch = reinterpret_cast<float*>(smem);                  // 64 floats
  bf16* xs = reinterpret_cast<bf16*>(smem + 256);                    // LN / PARTS: [M][K]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n0 = (bid * nw + w) * R;
  const bf16* wr[R];
#pragma unroll
  for (int r = 0; r < R; r++) wr[r] = W + (size_t)min(n0 + r, N - 1) * K;
  // lane j = r * MM + m stores (row r, token m) in the epilogue; its operands go out first
  const int er = lane / MM, em = lane % MM;
  const EpiPre pre = epi_prefetch<bf16>(ep, em, n0 + er, lane < R * MM && em < M && n0 + er < N);
  // LN / PARTS: the activation loads are issued first, then the first U chunks of every weight
  // row, then the prologue math runs on the activations (their loads are the oldest, so waiting
  // for them does not wait for the weights) while the weight stream is in flight
  float4 xv[LN ? MM : 1][4];
  float xc[LN ? MM : 1];
  uint2 gb[4][2];
  if constexpr (LN) {
    if (threadIdx.x < 256) ln_rows_load<MM>(ln, M, K, xv, xc, gb);
  }
  int eid[XM == X_EMB ? MM : 1];
  uint2 egb[4][2];
  if constexpr (XM == X_EMB) emb_rows_prefetch<MM>(ln, M, K, eid, egb, gb);
  const int kq = K >> 2, ngroups = M * kq;  // PARTS: 4-column groups of all rows
  PartsRegs pr[XM == X_PARTS ? kPartsPre : 1];
  // plain loads after a kernel boundary; sc1 loads (L2-coherent across XCDs) for partials of the same launch
  auto pld1 = [wait](const float* p, size_t i) {
    if (wait) return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(p), (uint32_t)(i * 4), 0, 16));
    return p[i];
  };
  auto pld4 = [wait](const float* p, size_t i) {
    if (wait)
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(attn_rsrc(p), (uint32_t)(i * 4), 0, 16));
    return *reinterpret_cast<const float4*>(p + i);
  };
  if constexpr (XM == X_PARTS) {
    if (!wait) {
#pragma unroll
      for (int it = 0; it < kPartsPre; it++) {
        const int g = min((int)threadIdx.x + it * (int)blockDim.x, ngroups - 1);
        attn_parts_load(pa, g / kq, (g % kq) * 4, pld1, pld4, pr[it]);
      }
    }
  }
  bf16x8 wv[U][R];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int k = min(u * 512 + lane * 8, K - 8);
#pragma unroll
    for (int r = 0; r < R; r++) wv[u][r] = wload<!(FL & 1)>(wr[r] + k);
  }
  const bf16* xg;
  int xstride;
  if constexpr (LN) {
    ln_rows_finish<MM>(ln, M, K, xv, xc, gb, xs, scratch);
    xg = xs; xstride = K;
  } else if constexpr (XM == X_EMB) {
    emb_rows_finish<MM>(ln, M, K, eid, egb, gb, xs, scratch);
    xg = xs; xstride = K;
  } else if constexpr (XM == X_PARTS) {
    if (wait) {  // the attention blocks of this launch: poll, then every partial load below is sc1
      if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(wait), 0, 0, 16) < target) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {
            __builtin_amdgcn_raw_buffer_store_b32(1u, attn_rsrc(wait), 8, 0, 16);
            break;
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < kPartsPre; it++) {
        const int g = min((int)threadIdx.x + it * (int)blockDim.x, ngroups - 1);
        attn_parts_load(pa, g / kq, (g % kq) * 4, pld1, pld4, pr[it]);
      }
    }
    auto put = [&](int g, const PartsRegs& r) {
      float o[4];
      attn_parts_combine(pa.nsplit, r, o);
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = (bf16)o[j];
      *reinterpret_cast<bf16x4*>(xs + (size_t)(g / kq) * K + (g % kq) * 4) = v;
    };
#pragma unroll
    for (int it = 0; it < kPartsPre; it++) {
      const int g = threadIdx.x + it * blockDim.x;
      if (g < ngroups) put(g, pr[it]);
    }
    for (int g = threadIdx.x + kPartsPre * blockDim.x; g < ngroups; g += blockDim.x) {  // wide rows: load as we go
      PartsRegs r;
      attn_parts_load(pa, g / kq, (g % kq) * 4, pld1, pld4, r);
      put(g, r);
    }
    __syncthreads();
    xg = xs; xstride = K;
  } else {
    xg = X; xstride = K;
  }
  BS_STAMP(1);
  float acc[R][MM];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int m = 0; m < MM; m++) acc[r][m] = 0.f;
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  for (int kb = 0; kb < K; kb += 512 * U) {
    if (kb) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = min(kb + u * 512 + lane * 8, K - 8);
#pragma unroll
        for (int r = 0; r < R; r++) wv[u][r] = wload<!(FL & 1)>(wr[r] + k);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int kk = kb + u * 512 + lane * 8;
      const bool live = kk < K;
      const int k = min(kk, K - 8);
#pragma unroll
      for (int m = 0; m < MM; m++) {
        bf16x8 xv;
        if constexpr (FL & 2) xv = (bf16x8){1, 1, 1, 1, 1, 1, 1, 1};
        else xv = *reinterpret_cast<const bf16x8*>(xg + (size_t)min(m, M - 1) * xstride + k);
        xv = live ? xv : zero8;
#pragma unroll
        for (int r = 0; r < R; r++) acc[r][m] = dot8(wv[u][r], xv, acc[r][m]);
      }
    }
  }
  BS_STAMP(2);
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int m = 0; m < MM; m++) acc[r][m] = wave_sum(acc[r][m]);
  epi_dispatch(ep.kind, [&](auto kc) {
    constexpr int EK = decltype(kc)::value;
    if constexpr (EK == EPI_ARGMAX) {
      // R = 4, 4 waves: a block owns one 16-column tile; lane (4*w + r) holds column n0+r
      float* tv = scratch;  // [16][MM] values
      __syncthreads();
      if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
          for (int m = 0; m < MM; m++) tv[(w * R + r) * MM + m] = acc[r][m];
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const int col = threadIdx.x & 15, m = threadIdx.x >> 4;  // 4 rows of 16 lanes: m < 4
        const int n = blockIdx.x * 16 + col;
        const float v = m < MM ? tv[col * MM + (m < MM ? m : 0)] : 0.f;
        argmax_tile16(ep, m, n, v, m < M && n < N, (N + 15) >> 4);
      }
    } else {
      if (lane < R * MM) {
        // lane j = r * MM + m takes (row r, token m); static register selection
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
          for (int m = 0; m < MM; m++) v = (lane == r * MM + m) ? acc[r][m] : v;
        const int n = n0 + er;
        if constexpr (FL & 4) {
          if (v == 12345.f) ep.keys[0] = 1;
        } else if (em < M && n < N) {
          epi_store_pre<bf16, EK>(ep, em, n, v, pre);
        }
      }
    }
  });
  BS_STAMP(3);
}

template <int R, int MM, int U, int XM, int FL = 0, int LB = 256>  // LB: threads the registers are bounded for
__global__ __launch_bounds__(LB) void gemv_rows_kernel(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                                         LnArgs ln, AttnParts pa, int M, int N, int K, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemv_rows_block<R, MM, U, XM, FL>(W, X, ln, pa, M, N, K, ep, blockIdx.x, smem, nullptr, 0u);
}

// ------------------------------------------------------------------------------------
// gemv_tiles: batched decode GEMV, 4 < M <= 16*MT (bf16 X [M][K], K % 64 == 0).  A block owns T
// 16-row weight tiles (16T output columns); its WAVES waves split K in 64-wide units.  Per unit a
// lane (r = lane & 15, g = lane >> 4) streams 32 contiguous bytes of weight row r of every tile
// (4 lanes x 32 B = one 128-B line per row) and the matching 32 bytes of activation row r of every
// m-tile, then runs 2 v_mfma_f32_16x16x32_bf16 per (tile, m-tile).  A and B take columns in the same
// permuted order (k-step j of a unit = columns g*16 + 8j .. +8 of lane g), which leaves every dot
// product unchanged.  The activation fragments are shared by the T tiles, so activation (L2)
// traffic is 1/T of a one-tile-per-block design's; the next unit's loads are in flight while this
// unit's MFMAs run.  Wave partials meet in LDS; the epilogue walks n fastest (coalesced stores,
// and 16 aligned lanes = one 16-column argmax tile).
// ------------------------------------------------------------------------------------
// Weight-only int8 (WT = int8_t): a lane's 16 weights of a unit are 16 bytes, converted in registers to
// two exact bf16x8 (|Q| <= 127; u = q ^ 0x80 through v_cvt_f32_ubyte*, minus 128) before the same MFMAs;
// the row scale is the epilogue's col_scale.  Half the streamed bytes of the bf16 tiles, no dequant pass.
__device__ __forceinline__ void q8x16_to_bf16(const u32x4v raw, bf16x8& lo, bf16x8& hi) {
  const uint32_t v[4] = {raw.x ^ 0x80808080u, raw.y ^ 0x80808080u, raw.z ^ 0x80808080u, raw.w ^ 0x80808080u};
#pragma unroll
  for (int i = 0; i < 2; i++) {
    bf16x8& o = i ? hi : lo;
    const uint32_t a = v[2 * i], b = v[2 * i + 1];
    // (float)(byte) lowers to v_cvt_f32_ubyte{0..3}
    o[0] = (bf16)((float)(a & 0xFF) - 128.f); o[1] = (bf16)((float)((a >> 8) & 0xFF) - 128.f);
    o[2] = (bf16)((float)((a >> 16) & 0xFF) - 128.f); o[3] = (bf16)((float)(a >> 24) - 128.f);
    o[4] = (bf16)((float)(b & 0xFF) - 128.f); o[5] = (bf16)((float)((b >> 8) & 0xFF) - 128.f);
    o[6] = (bf16)((float)((b >> 16) & 0xFF) - 128.f); o[7] = (bf16)((float)(b >> 24) - 128.f);
  }
}

// Tile GEMV epilogue: every wave's partial tiles meet in LDS (`red`, [WAVES][T*16][MT*16+1]); split-K
// blocks publish write-through partials and the last arriver sums them in split order; then the epilogue.
template <int T, int MT, int WAVES>
__device__ __forceinline__ void tiles_epilogue(const f32x4 (&acc)[T][MT], float* red, int M, int N, int n0,
                                               const Epi& ep) {
  constexpr int RS = MT * 16 + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int KS = gridDim.y, ks = blockIdx.y;
  // D[row = 4g + i (n)][col = r (m)]
  float* rw = red + (size_t)w * (T * 16) * RS;
#pragma unroll
  for (int t = 0; t < T; t++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int i = 0; i < 4; i++) rw[(t * 16 + 4 * g + i) * RS + mt * 16 + r] = acc[t][mt][i];
  __syncthreads();
  const int ntiles = (N + 15) >> 4;
  constexpr int TOTAL = T * 16 * MT * 16, NTH = WAVES * 64;
  constexpr int ITER = (TOTAL + NTH - 1) / NTH;
  float vs[ITER];
#pragma unroll
  for (int it = 0; it < ITER; it++) {
    const int idx = it * NTH + threadIdx.x;
    const int nl = idx % (T * 16), ml = idx / (T * 16);
    float v = 0.f;
    if (idx < TOTAL) {
#pragma unroll
      for (int ww = 0; ww < WAVES; ww++) v += red[((size_t)ww * (T * 16) + nl) * RS + ml];
    }
    vs[it] = v;
  }
  if (KS > 1) {
    // publish this block's partial tile (write-through), take a ticket; the last of the KS blocks
    // of this column range sums the KS partials in split order (deterministic) and runs the epilogue
#pragma unroll
    for (int it = 0; it < ITER; it++) {
      const int idx = it * NTH + threadIdx.x;
      const int nl = idx % (T * 16), ml = idx / (T * 16), n = n0 + nl;
      if (idx < TOTAL && ml < M && n < N)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vs[it]), attn_rsrc(ep.sk_ws),
                                              (uint32_t)(((size_t)ks * M + ml) * N + n) * 4, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int sk_last;
    __syncthreads();
    if (threadIdx.x == 0) {
      typedef __attribute__((address_space(1))) unsigned gu32;
      const unsigned old = __hip_atomic_fetch_add((gu32*)(ep.sk_tickets + blockIdx.x), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      sk_last = old == (unsigned)(KS - 1);
      if (sk_last) __hip_atomic_store((gu32*)(ep.sk_tickets + blockIdx.x), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!sk_last) return;
#pragma unroll
    for (int it = 0; it < ITER; it++) {
      const int idx = it * NTH + threadIdx.x;
      const int nl = idx % (T * 16), ml = idx / (T * 16), n = n0 + nl;
      float v = 0.f;
      if (idx < TOTAL && ml < M && n < N) {
        for (int k2 = 0; k2 < KS; k2++)
          v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(ep.sk_ws),
                                                                    (uint32_t)(((size_t)k2 * M + ml) * N + n) * 4, 0, 16));
      }
      vs[it] = v;
    }
  }
  epi_dispatch(ep.kind, [&](auto kc) {
    constexpr int EK = decltype(kc)::value;
#pragma unroll
    for (int it = 0; it < ITER; it++) {  // uniform trip count: argmax needs every lane
      const int idx = it * NTH + threadIdx.x;
      const int nl = idx % (T * 16), ml = idx / (T * 16);
      const int n = n0 + nl;
      epi_apply<bf16, EK>(ep, ml, n, vs[it], idx < TOTAL && ml < M && n < N, ntiles);
    }
  });
}

template <int T, int MT, int WAVES, typename WT = bf16, int PD = 2, bool IL = false, int J = 2>
__global__ __launch_bounds__(WAVES * 64) void gemv_tiles_kernel(const WT* __restrict__ W, const bf16* __restrict__ X,
                                                                int M, int N, int K, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RS = MT * 16 + 1;  // padded LDS row: [n][m]
  constexpr int KU = 32 * J;       // K columns per unit: J MFMA k-steps; lane g holds 8J contiguous columns
  float* red = reinterpret_cast<float*>(smem);  // [WAVES][T * 16][RS]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (T * 16);
  // split-K: block (x, ks) takes units [ks * upb, (ks + 1) * upb), its waves split those
  const int KS = gridDim.y, ks = blockIdx.y;
  const int units_all = K / KU, upb = (units_all + KS - 1) / KS;
  const int ub0 = min(units_all, ks * upb), units = min(units_all, ub0 + upb) - ub0;
  const int per = (units + WAVES - 1) / WAVES;
  const int u0 = ub0 + min(units, w * per), u1 = ub0 + min(units, w * per + per);
  const WT* wp[T];
#pragma unroll
  for (int t = 0; t < T; t++) wp[t] = W + (size_t)min(n0 + t * 16 + r, N - 1) * K + g * 8 * J;
  const bf16* xp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) xp[mt] = X + (size_t)min(mt * 16 + r, M - 1) * K + g * 8 * J;
  f32x4 acc[T][MT];
#pragma unroll
  for (int t = 0; t < T; t++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++) acc[t][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // a unit's raw operands: per tile J bf16x8 (bf16) or J / 2 16-B int8 words (converted where used); k-step
  // j of a unit takes columns 8j .. 8j + 8 of every lane's run, in A (weights) and B (activations) alike
  constexpr bool Q8 = sizeof(WT) == 1;
  constexpr int NW = Q8 ? J / 2 : J;
  typedef u32x4v RawW[NW];
  auto load = [&](int u, RawW (&aa)[T], bf16x8 (&bb)[MT][J]) {
    const size_t o = (size_t)u * KU;
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
      for (int h = 0; h < NW; h++)
        aa[t][h] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(wp[t] + o + h * 16 / sizeof(WT)));
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int j = 0; j < J; j++) bb[mt][j] = *reinterpret_cast<const bf16x8*>(xp[mt] + o + 8 * j);
  };
  // Register ring of PD units: slot p holds unit i + p of the wave's list; after its MFMAs the slot is
  // refilled with unit i + p + PD.  The loads are unconditional (clamped: a re-read of the wave's last unit
  // is unused) so the compiler counts them with vmcnt(N) and keeps PD - 1 units in flight behind the MFMAs.
  // IL: wave w takes units w, w + WAVES, ... of its block's range (the CU's waves stream adjacent K
  // columns of the same rows); otherwise a contiguous range per wave
  const int nu = IL ? (units > w ? (units - w + WAVES - 1) / WAVES : 0) : u1 - u0;
  auto unit = [&](int i) { return IL ? ub0 + w + min(i, nu - 1) * WAVES : u0 + min(i, nu - 1); };
  if (nu > 0) {
    RawW a[PD][T];
    bf16x8 b[PD][MT][J];
#pragma unroll
    for (int p = 0; p < PD; p++) load(unit(p), a[p], b[p]);
    for (int i = 0; i < nu; i += PD) {
#pragma unroll
      for (int p = 0; p < PD; p++) {
        if (i + p < nu) {  // wave-uniform
          bf16x8 w8[T][J];
#pragma unroll
          for (int t = 0; t < T; t++) {
#pragma unroll
            for (int h = 0; h < NW; h++) {
              if constexpr (Q8) q8x16_to_bf16(a[p][t][h], w8[t][2 * h], w8[t][2 * h + 1]);
              else w8[t][h] = __builtin_bit_cast(bf16x8, a[p][t][h]);
            }
          }
#pragma unroll
          for (int j = 0; j < J; j++)
#pragma unroll
            for (int t = 0; t < T; t++)
#pragma unroll
              for (int mt = 0; mt < MT; mt++)
                acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w8[t][j], b[p][mt][j], acc[t][mt], 0, 0, 0);
        }
        load(unit(i + p + PD), a[p], b[p]);
      }
    }
  }
  tiles_epilogue<T, MT, WAVES>(acc, red, M, N, n0, ep);
}

// ------------------------------------------------------------------------------------
// gemv_ldsw4: the batched-decode GEMV with the weight stream read as the rows GEMV reads it.  The MFMA
// operand layout wants 16 rows x 64 B per load instruction, which streamed at ~4.2 TB/s in gemv_tiles
// (profiles/r02_tiles_sweep.txt); here a load instruction reads one 128-B line of each of 8 rows, the wave
// writes its stage (T*16 rows x 64 columns) to a private LDS region (16-B chunks XOR-swizzled by row) and
// reads the A fragments from there.  Every wave covers all T tiles of its block and a K part (waves split
// K, as in gemv_tiles), so one wave's activation fragments serve T weight tiles; the next stage's weights
// and activations are in flight (registers) while the current stage is computed.  bf16 weights.
// ------------------------------------------------------------------------------------
// 8 int8 weights (8 bytes) -> bf16x8 exactly (|q| <= 127): u = q ^ 0x80 through v_cvt_f32_ubyte*, minus 128
__device__ __forceinline__ bf16x8 q8x8_to_bf16(const uint2 raw) {
  const uint32_t a = raw.x ^ 0x80808080u, b = raw.y ^ 0x80808080u;
  bf16x8 o;
  o[0] = (bf16)((float)(a & 0xFF) - 128.f); o[1] = (bf16)((float)((a >> 8) & 0xFF) - 128.f);
  o[2] = (bf16)((float)((a >> 16) & 0xFF) - 128.f); o[3] = (bf16)((float)(a >> 24) - 128.f);
  o[4] = (bf16)((float)(b & 0xFF) - 128.f); o[5] = (bf16)((float)((b >> 8) & 0xFF) - 128.f);
  o[6] = (bf16)((float)((b >> 16) & 0xFF) - 128.f); o[7] = (bf16)((float)(b >> 24) - 128.f);
  return o;
}

// WT = bf16 (KC = 64 columns = 128 B per row per stage) or int8_t (KC = 128 columns = 128 B; each A fragment
// is 8 bytes converted in registers, the row scale applied by the epilogue's col_scale).
// PD: stages in flight per wave (register ring): 2, or 3 when a wave's K part is exactly 3 stages (the
// bloom-1b1 widths), so every load of the wave is issued before its first stage waits.
// LNS > 0 (bf16 weights, MT = 1, one K split): X is LN(ln.x) -- the LayerNorm runs in the prologue.  A wave's K
// part is exactly LNS stages; its lanes load their fp32 activations of every stage (row r, the columns of their
// B fragments) behind the first weight stages, take the shifted sums of ln_rows_wave_kernel over them, and the
// 8 waves' sums meet in LDS (one barrier) -- the waves together cover the whole row.  The normalised bf16
// fragments stay in registers for the whole K loop (no activation loads in it).
template <int T, int WAVES, int MT, typename WT = bf16, int PD = 2, int LNS = 0>
__global__ __launch_bounds__(WAVES * 64) void gemv_ldsw4_kernel(const WT* __restrict__ W, const bf16* __restrict__ X,
                                                               int M, int N, int K, Epi ep, LnArgs ln) {
  constexpr int RB = 128, KC = RB / (int)sizeof(WT);  // bytes / columns of one row per stage
  constexpr int CPR = RB / 16, RPI = 64 / CPR, ROWS = T * 16, NI = ROWS / RPI, KSTEP = KC / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  char* wl = smem + (size_t)w * ROWS * RB;
  float* red = reinterpret_cast<float*>(smem + (size_t)WAVES * ROWS * RB);
  const int n0 = blockIdx.x * ROWS;
  const int KS = gridDim.y, ks = blockIdx.y;
  const int kw = K / (KS * WAVES);  // host: a multiple of KC
  const int kbeg = ks * (K / KS) + w * kw, nst = kw / KC;
  const int lr = lane / CPR, lc = lane % CPR;
  const int rows_ok = min(ROWS, N - n0);
  const WT* wsrc = W + (size_t)min(n0 + lr, N - 1) * K + kbeg + lc * (16 / (int)sizeof(WT));
  const size_t wstep = (size_t)RPI * K;
  auto swz = [](int row, int byte) {  // 16-B chunks XOR-swizzled by row
    return row * RB + ((((byte >> 4) ^ (row & (CPR - 1)))) << 4) + (byte & 15);
  };
  const bf16* xsrc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) xsrc[mt] = X + (size_t)min(mt * 16 + r, M - 1) * K + kbeg + g * 8;
  u32x4v wr[PD][NI];
  bf16x8 xr[PD][MT][KSTEP];
  auto load = [&](int st, u32x4v (&ww)[NI], bf16x8 (&xx)[MT][KSTEP]) {
    const size_t o = (size_t)st * KC;
#pragma unroll
    for (int i = 0; i < NI; i++) {
      const WT* src = (RPI * i + lr < rows_ok) ? wsrc + i * wstep : wsrc;
      ww[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(src + o));
    }
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int j = 0; j < KSTEP; j++)  // B rows past M are never stored: no load (no duplicate activation traffic)
        xx[mt][j] = mt * 16 + r < M ? *reinterpret_cast<const bf16x8*>(xsrc[mt] + o + 32 * j) : (bf16x8){};
  };
  f32x4 acc[T][MT];
#pragma unroll
  for (int t = 0; t < T; t++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++) acc[t][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int b, int st) {
    const int nb = (b + PD - 1) % PD;  // the ring slot of stage st + PD - 1
    if (st + PD - 1 < nst) load(st + PD - 1, wr[nb], xr[nb]);
#pragma unroll
    for (int i = 0; i < NI; i++) *reinterpret_cast<u32x4v*>(&wl[swz(RPI * i + lr, lc * 16)]) = wr[b][i];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < KSTEP; j++)
#pragma unroll
      for (int t = 0; t < T; t++) {
        // k-step j: columns 32j .. 32j + 32 of the stage; lane g takes 8g .. 8g + 8
        bf16x8 af;
        if constexpr (sizeof(WT) == 1) af = q8x8_to_bf16(*reinterpret_cast<const uint2*>(&wl[swz(t * 16 + r, 32 * j + 8 * g)]));
        else af = *reinterpret_cast<const bf16x8*>(&wl[swz(t * 16 + r, 64 * j + 16 * g)]);
#pragma unroll
        for (int mt = 0; mt < MT; mt++) acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, xr[b][mt][j], acc[t][mt], 0, 0, 0);
      }
    __builtin_amdgcn_wave_barrier();
  };
  if constexpr (LNS > 0) {
    static_assert(sizeof(WT) == 2, "LN prologue: bf16 weights");
    auto loadw = [&](int st, u32x4v (&ww)[NI]) {
      const size_t o = (size_t)st * KC;
#pragma unroll
      for (int i = 0; i < NI; i++) {
        const WT* src = (RPI * i + lr < rows_ok) ? wsrc + i * wstep : wsrc;
        ww[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(src + o));
      }
    };
    // rows 16 mt + r (< M; rows past M are never stored and load nothing), columns kbeg + KC * st + 32 j + 8 g .. + 8:
    // this lane's B fragments.  gamma / beta of the wave's K part go through LDS once (16 B per lane, 2 x KC x LNS x
    // 2 B per wave) and are read back as broadcasts, so the block reads them once per wave, not once per B row.
    // (dead lanes: an offset past the buffer's records -- the load returns 0 and moves no bytes)
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(ln.x), (short)0, (int)((((size_t)(M - 1) * ln.row_stride + ln.row_offset) * K + K) * 4), 0x00020000);
    uint32_t xoff[MT];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
      xoff[mt] = mt * 16 + r < M ? (uint32_t)(((size_t)(mt * 16 + r) * ln.row_stride + ln.row_offset) * K * 4) : 0x80000000u;
    float4 xf[MT][LNS][KSTEP][2];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int st = 0; st < LNS; st++)
#pragma unroll
        for (int j = 0; j < KSTEP; j++) {
          const uint32_t col = (uint32_t)(kbeg + st * KC + 32 * j + 8 * g) * 4;
          xf[mt][st][j][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff[mt] + col, 0, 0));
          xf[mt][st][j][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff[mt] + col + 16, 0, 0));
        }
    float c[MT];
#pragma unroll
    for (int mt = 0; mt < MT; mt++) c[mt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, xoff[mt], 0, 0));
    constexpr int GB = LNS * KC * 2 / 16;  // 16-B pieces of the wave's gamma (and of its beta)
    constexpr int GI = (2 * GB + 63) / 64;
    float* sred = red + WAVES * (T * 16) * (MT * 16 + 1);  // [WAVES][16 MT rows][2], after the epilogue's area
    char* gbl = reinterpret_cast<char*>(sred + WAVES * 32 * MT) + (size_t)w * GB * 32;
    u32x4v gtmp[GI];
#pragma unroll
    for (int it = 0; it < GI; it++) {
      const int i = min(it * 64 + lane, 2 * GB - 1);
      gtmp[it] = *reinterpret_cast<const u32x4v*>((i < GB ? ln.gamma : ln.beta) + kbeg + (i % GB) * 8);
    }
    // the weight stream goes out behind the activations (loads return in order: waiting for the activations
    // leaves the weights in flight), every stage of the wave's K part at once when the ring holds them all
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < PD; p++)
      if (p < LNS) loadw(p, wr[p]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < GI; it++)
      if (it * 64 + lane < 2 * GB) *reinterpret_cast<u32x4v*>(gbl + (it * 64 + lane) * 16) = gtmp[it];
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int st = 0; st < LNS; st++)
#pragma unroll
        for (int j = 0; j < KSTEP; j++)
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const float4 v = xf[mt][st][j][h];
            const float d0 = v.x - c[mt], d1 = v.y - c[mt], d2 = v.z - c[mt], d3 = v.w - c[mt];
            a1 += (d0 + d1) + (d2 + d3);
            a2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
          }
      a1 += __shfl_xor(a1, 16, 64); a1 += __shfl_xor(a1, 32, 64);
      a2 += __shfl_xor(a2, 16, 64); a2 += __shfl_xor(a2, 32, 64);
      if (g == 0) { sred[(w * 16 * MT + mt * 16 + r) * 2] = a1; sred[(w * 16 * MT + mt * 16 + r) * 2 + 1] = a2; }
    }
    __syncthreads();
    const float invk = 1.0f / (float)K;
    bf16x8 xn[MT][LNS][KSTEP];
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ww++) {
        t1 += sred[(ww * 16 * MT + mt * 16 + r) * 2];
        t2 += sred[(ww * 16 * MT + mt * 16 + r) * 2 + 1];
      }
      t1 *= invk; t2 *= invk;
      const float mean = c[mt] + t1, rstd = 1.0f / sqrtf(fmaxf(t2 - t1 * t1, 0.f) + ln.eps);
#pragma unroll
      for (int st = 0; st < LNS; st++)
#pragma unroll
        for (int j = 0; j < KSTEP; j++) {
          float4 g0, g1, b0, b1;
          const int pc = (st * KC + 32 * j + 8 * g) / 8;  // 16-B piece of the wave's K part
          const u32x4v gv = *reinterpret_cast<const u32x4v*>(gbl + pc * 16);
          const u32x4v bv = *reinterpret_cast<const u32x4v*>(gbl + (GB + pc) * 16);
          bf16x4_to_f32(make_uint2(gv.x, gv.y), g0);
          bf16x4_to_f32(make_uint2(gv.z, gv.w), g1);
          bf16x4_to_f32(make_uint2(bv.x, bv.y), b0);
          bf16x4_to_f32(make_uint2(bv.z, bv.w), b1);
          const float4 v0 = xf[mt][st][j][0], v1 = xf[mt][st][j][1];
          bf16x8 o;
          o[0] = (bf16)((v0.x - mean) * rstd * g0.x + b0.x); o[1] = (bf16)((v0.y - mean) * rstd * g0.y + b0.y);
          o[2] = (bf16)((v0.z - mean) * rstd * g0.z + b0.z); o[3] = (bf16)((v0.w - mean) * rstd * g0.w + b0.w);
          o[4] = (bf16)((v1.x - mean) * rstd * g1.x + b1.x); o[5] = (bf16)((v1.y - mean) * rstd * g1.y + b1.y);
          o[6] = (bf16)((v1.z - mean) * rstd * g1.z + b1.z); o[7] = (bf16)((v1.w - mean) * rstd * g1.w + b1.w);
          xn[mt][st][j] = o;
        }
    }
#pragma unroll
    for (int st = 0; st < LNS; st++) {
      const int b = st % PD;
#pragma unroll
      for (int i = 0; i < NI; i++) *reinterpret_cast<u32x4v*>(&wl[swz(RPI * i + lr, lc * 16)]) = wr[b][i];
      if (st + PD < LNS) loadw(st + PD, wr[b]);  // a ring shallower than the K part: refill the slot just staged
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < KSTEP; j++)
#pragma unroll
        for (int t = 0; t < T; t++) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(&wl[swz(t * 16 + r, 64 * j + 16 * g)]);
#pragma unroll
          for (int mt = 0; mt < MT; mt++)
            acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, xn[mt][st][j], acc[t][mt], 0, 0, 0);
        }
      __builtin_amdgcn_wave_barrier();
    }
  } else if (nst > 0) {
#pragma unroll
    for (int p = 0; p < PD - 1; p++)
      if (p < nst) load(p, wr[p], xr[p]);
    for (int st = 0; st < nst; st += PD) {
#pragma unroll
      for (int p = 0; p < PD; p++)
        if (st + p < nst) stage(p, st + p);
    }
  }
  tiles_epilogue<T, MT, WAVES>(acc, red, M, N, n0, ep);
}

template <int T, int WAVES, int MT, typename WT>
static void gemv_ldsw4_launch(const bf16* X, const WT* W, int M, int N, int K, int KS, const Epi& ep, hipStream_t s) {
  const size_t shm = (size_t)WAVES * T * 16 * 128 + sizeof(float) * WAVES * (T * 16) * (MT * 16 + 1);
  const int blocks = (N + T * 16 - 1) / (T * 16);
  constexpr int KC = 128 / (int)sizeof(WT);
  if constexpr (sizeof(WT) == 2) {
    if (K / (KS * WAVES * KC) == 3) {
      gemv_ldsw4_kernel<T, WAVES, MT, WT, 3><<<dim3(blocks, KS), WAVES * 64, shm, s>>>(W, X, M, N, K, ep, LnArgs{});
      return;
    }
  }
  gemv_ldsw4_kernel<T, WAVES, MT, WT, 2><<<dim3(blocks, KS), WAVES * 64, shm, s>>>(W, X, M, N, K, ep, LnArgs{});
}

// LN-fused gemv_ldsw4 (bf16, M <= 16, one K split): a wave's K part is K / (8 * 64) stages, 2..5 supported.  (Two
// m-tiles, 16 < M <= 32, measured slower than the LayerNorm launch + the plain GEMV: bloom-1b1 QKV at M = 32 12.9 vs
// 2.9 + 7.8 us, decode B = 32 21708 -> 20598 tok/s, profiles/r05_ln_prologue_ab.txt -- the fp32 rows of 32 tokens
// are twice the bf16 activation bytes the plain GEMV streams.)
template <int T>
static bool gemv_ldsw4_ln_launch(const LnArgs& ln, const bf16* W, int M, int N, int K, const Epi& ep, hipStream_t s) {
  constexpr int WAVES = 8;
  const int nst = K / (WAVES * 64);
  const int mt = 1;
  // where the fused LayerNorm beats the LayerNorm launch + plain tile GEMV (round 6, profiles/r06_lns_ab.txt): rows of
  // K <= 1024 at every M (bloom-560m +3-7 %), K <= 1536 up to M = 8 (bloom-1b1 +1-2 %; M = 16 -1 %), not at bloom-3b's
  // K = 2560 (-0.3 .. -4 %: every block loads all M fp32 rows).  BS_LNS_MAX_M (read once) replaces the rule.
  static const int lns_max_m = [] {
    const char* e = getenv("BS_LNS_MAX_M");
    return e ? atoi(e) : -1;
  }();
  if (lns_max_m >= 0 ? M > lns_max_m : !(K <= 1024 || (K <= 1536 && M <= 8))) return false;
  if (M > 16 || K % (WAVES * 64) || nst < 2 || nst > 5) return false;
  // the activation descriptor's byte size and the per-row offsets are 32-bit: rows that reach 2^31 bytes (a long
  // lm_head row stride) take the LayerNorm launch instead
  if ((size_t)((size_t)(M - 1) * ln.row_stride + ln.row_offset + 1) * K * 4 >= ((size_t)1 << 31)) return false;
  // weight stages, wave partials, the statistics' exchange, each wave's gamma / beta (2 x nst x 64 x 2 B)
  const size_t shm = (size_t)WAVES * T * 16 * 128 + sizeof(float) * WAVES * (T * 16) * (mt * 16 + 1) +
                     sizeof(float) * WAVES * 32 * mt + (size_t)WAVES * nst * 64 * 4;
  const int blocks = (N + T * 16 - 1) / (T * 16);
  auto go = [&](auto mc, auto pc, auto lc) {
    constexpr int MTc = decltype(mc)::value, PDc = decltype(pc)::value, LNSc = decltype(lc)::value;
    gemv_ldsw4_kernel<T, WAVES, MTc, bf16, PDc, LNSc><<<blocks, WAVES * 64, shm, s>>>(W, nullptr, M, N, K, ep, ln);
  };
  // ring = the whole K part (every weight stage in flight behind the activations) while T x stages <= 12 keeps the
  // kernel spill-free (ISA metadata), else 2 stages
  switch (nst) {
    case 2: go(EpiKindC<1>{}, EpiKindC<2>{}, EpiKindC<2>{}); break;
    case 3: go(EpiKindC<1>{}, EpiKindC<3>{}, EpiKindC<3>{}); break;
    case 4: go(EpiKindC<1>{}, EpiKindC<T <= 3 ? 4 : 2>{}, EpiKindC<4>{}); break;
    default: go(EpiKindC<1>{}, EpiKindC<T <= 2 ? 5 : 2>{}, EpiKindC<5>{}); break;
  }
  return true;
}

template <int T, int MT, int WAVES, typename WT = bf16>
static void gemv_tiles_launch(const bf16* X, const WT* W, int M, int N, int K, int KS, const Epi& ep, hipStream_t s) {
  const size_t shm = sizeof(float) * WAVES * (T * 16) * (MT * 16 + 1);
  const int blocks = (N + T * 16 - 1) / (T * 16);
  const dim3 g(blocks, KS);
  // interleaved units: +12 % on bloom-7b1 B = 32 decode over contiguous unit ranges per wave
  // (profiles/r02_tiles_sweep.txt); deeper register rings (PD 3, 4) and 4-k-step units measured slower
  gemv_tiles_kernel<T, MT, WAVES, WT, 2, true><<<g, WAVES * 64, shm, s>>>(W, X, M, N, K, ep);
}

// Shape choice: the BLOOM shapes take the fastest (tiles, K splits, waves) of the
// tools/gemv_probe.hip PROBE_SWEEP measurement (profiles/r01_gemv_sweep.log), per m-tile count;
// other shapes: 2 tiles (4 from N >= 16384), K split until >= 192 blocks while each split keeps
// >= 8 units, 8 waves when every wave gets >= 2 units.
// bloom-3b fc1/fc2 and bloom-7b1 QKV/fc2 (M <= 16) re-swept for gemv_ldsw4 (whose K parts must divide
// K: 3b fc1 had fallen back to gemv_tiles): 3b B=8 3031 -> 3927 tok/s, B=32 8124 -> 10624; 7b1 B=16 QKV
// 21.2 -> 18.3 us, fc2 26.8 -> 24.6 us; 1b1 dense at M > 16 (1, 1): 8.9 -> 6.8 us; 560m (h = 1024) rows added (B=32 QKV 8.1 -> 5.6 us;
// profiles/r02_tiles_sweep.txt)
struct TileCfg { int N, K, T1, KS1, W1, T2, KS2, W2; };  // (T, KS, waves) for M <= 16 and M <= 32
static const TileCfg kTileTable[] = {
  {3072, 1024, 1, 1, 8, 1, 1, 8},    {1024, 1024, 1, 1, 8, 1, 1, 8},   {4096, 1024, 2, 1, 8, 2, 1, 8},
  {1024, 4096, 1, 1, 8, 1, 4, 8},
  {4608, 1536, 2, 1, 8, 2, 1, 8},    {1536, 1536, 1, 1, 8, 1, 1, 8},   {6144, 1536, 2, 1, 8, 2, 1, 8},
  {1536, 6144, 1, 2, 8, 1, 2, 8},    {7680, 2560, 2, 1, 8, 2, 1, 8},   {2560, 2560, 1, 1, 8, 1, 1, 8},
  {10240, 2560, 3, 1, 8, 3, 1, 8},   {2560, 10240, 2, 2, 8, 2, 5, 8},  {12288, 4096, 3, 1, 8, 3, 1, 8},
  {4096, 4096, 1, 1, 8, 2, 2, 8},    {16384, 4096, 4, 1, 8, 4, 1, 8},  {4096, 16384, 2, 2, 8, 2, 2, 8},
};

// Token counts the batched tile GEMV (gemv_ldsw4) takes for plain and LayerNorm-fused GEMVs: M >= 3, and M = 2 on
// K >= 2560 (bloom-3b / 7b1 widths); below, the rows GEMV.  Round 6 (tools/gpu_r6w.sh, profiles/r06_tiles_min_m_ab.txt):
// M = 3..4 had gone to the rows GEMV (whose time grows with M: bloom-1b1 fc2 7.0 -> 10.9 us from M = 1 to 4) or the
// old gemv_mfma; on the tile GEMV decode at B = 3 / 4 runs +28-38 % (bloom-1b1 B = 4 3122 -> 4140 tok/s, 7b1
// 999 -> 1351), B = 2 +3 % (3b) / +11 % (7b1), while bloom-1b1 B = 2 keeps the rows GEMV (-4 % on tiles).
// BS_TILES_MIN_M (read once) replaces the rule by a plain threshold for A/B runs.
static bool tiles_take(int M, int K) {
  static const int v = [] {
    const char* e = getenv("BS_TILES_MIN_M");
    const int m = e ? atoi(e) : 0;
    return m >= 2 && m <= 33 ? m : 0;
  }();
  if (v) return M >= v;
  return M >= 3 || (M == 2 && K >= 2560);
}

// Largest token count of the batched tile GEMV: 64 (bf16 weights, four m-tiles, 32 < M <= 64: short prefills, which
// the prefill GEMMs' 128-row tiles serve with most of each tile and most CUs idle), or 32 with BS_TILES_MAX_M=32
// (A/B knob, read once).
static int tiles_max_m() {
  static const int v = [] {
    const char* e = getenv("BS_TILES_MAX_M");
    return e && atoi(e) == 32 ? 32 : 64;
  }();
  return v;
}

// ln != nullptr (bf16): X = LN(ln->x) fused into gemv_ldsw4's prologue when the shape takes one K split of
// 2..5 stages per wave and M <= 16; otherwise returns false and the caller normalises first.
// 32 < M <= 64 (bf16, no LN): gemv_ldsw4 with four m-tiles where the table's tile count is <= 3 (the LDS of the wave
// partials), else false (the prefill GEMM).
template <typename WT = bf16>
static bool gemv_tiles_dispatch(const bf16* x, const WT* w, int M, int N, int K, const Epi& ep, hipStream_t s,
                                const LnArgs* ln = nullptr) {
  if (!tiles_take(M, K) || M > 64 || (K % 64) != 0) return false;
  const bool four = M > 32;
  // four m-tiles only on the long-K shapes (fc2, K = 4N), whose prefill GEMM has few output tiles: bloom-1b1 fc2 at 64
  // tokens 22.4 -> 18.1 us, while QKV / fc1 (10.8 / 9.2 -> 12.2 us) and dense (8.3 -> 9.6 us) keep the GEMM's
  // 64 x 32 tiles (profiles/r06_tiles_four_m_ab.txt)
  if (four && (sizeof(WT) != 2 || ln || M > tiles_max_m() || K < 4 * N)) return false;
  const int units = K / 64;
  int T = N >= 16384 ? 4 : 2, KS = 1, WV = 0;
  for (const TileCfg& c : kTileTable)
    if (c.N == N && c.K == K) {
      T = M > 16 ? c.T2 : c.T1; KS = M > 16 ? c.KS2 : c.KS1; WV = M > 16 ? c.W2 : c.W1;
    }
  const int blocks = (N + T * 16 - 1) / (T * 16);
  const bool sk_ok = ep.sk_ws && ep.sk_tickets && blocks <= ep.sk_ntickets;
  if (WV == 0) {  // not in the table
    if (sk_ok)
      while (blocks * KS < 192 && units / (KS * 2) >= 8 && (size_t)KS * 2 * M * N <= ep.sk_cap) KS *= 2;
    WV = (units + KS - 1) / KS >= 16 ? 8 : 4;
  }
  if (KS > 1 && (!sk_ok || (size_t)KS * M * N > ep.sk_cap)) KS = 1;  // no workspace: no split
  const bool two = M > 16;
  {
    // gemv_ldsw4 at the table's (T, KS) (bloom-7b1 B=32: qkv 29.7 -> 21.3 us, dense 15.8 -> 12.5, fc1
    // 36.4 -> 25.6, fc2 43.1 -> 32.0; decode steps: 7b1 B=16 +11 %, 3b B=8 +35 %, 1b1 B=8 +32 % over
    // gemv_tiles; profiles/r02_tiles_sweep.txt).  gemv_tiles takes the shapes whose K parts do not divide K.
    constexpr int KC = 128 / (int)sizeof(WT);
    if (ln) {
      if constexpr (sizeof(WT) == 2) {
        if (KS != 1 || T > 4) return false;
        if (T == 4) return gemv_ldsw4_ln_launch<4>(*ln, w, M, N, K, ep, s);
        if (T == 3) return gemv_ldsw4_ln_launch<3>(*ln, w, M, N, K, ep, s);
        if (T == 2) return gemv_ldsw4_ln_launch<2>(*ln, w, M, N, K, ep, s);
        return gemv_ldsw4_ln_launch<1>(*ln, w, M, N, K, ep, s);
      }
      return false;
    }
    if (four && (T > 3 || K % (KS * 8 * KC) != 0)) return false;
    if (T <= 4 && K % (KS * 8 * KC) == 0) {
      auto go4 = [&](auto tc) {
        constexpr int TT = decltype(tc)::value;
        if constexpr (TT <= 3 && sizeof(WT) == 2) {
          if (four) {
            gemv_ldsw4_launch<TT, 8, 4, WT>(x, w, M, N, K, KS, ep, s);
            return;
          }
        }
        if (two) gemv_ldsw4_launch<TT, 8, 2, WT>(x, w, M, N, K, KS, ep, s);
        else gemv_ldsw4_launch<TT, 8, 1, WT>(x, w, M, N, K, KS, ep, s);
      };
      if (T == 4) go4(EpiKindC<4>{});
      else if (T == 3) go4(EpiKindC<3>{});
      else if (T == 2) go4(EpiKindC<2>{});
      else go4(EpiKindC<1>{});
      return true;
    }
  }
  auto go = [&](auto tc, auto wc) {
    constexpr int TT = decltype(tc)::value, WW = decltype(wc)::value;
    if (two) gemv_tiles_launch<TT, 2, WW, WT>(x, w, M, N, K, KS, ep, s);
    else gemv_tiles_launch<TT, 1, WW, WT>(x, w, M, N, K, KS, ep, s);
  };
  auto gw = [&](auto tc) {
    if (WV == 4) go(tc, EpiKindC<4>{});
    else go(tc, EpiKindC<8>{});
  };
  if (T == 4) gw(EpiKindC<4>{});
  else if (T == 3) gw(EpiKindC<3>{});
  else if (T == 2) gw(EpiKindC<2>{});
  else gw(EpiKindC<1>{});
  return true;
}

// ------------------------------------------------------------------------------------
// gemm_mfma: C = X[M][K] . W[N][K]^T, BM x BN tile per 256-thread block (2x2 waves),
// BK = 32, LDS double buffer with register staging, rows padded by 8 elements.
// A = X tile (rows = m), B = W^T tile (cols = n): D[row = m][col = n].
// ------------------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                        int M, int N, int K, Epi ep) {
  constexpr int BK = 32, LDK = BK + 8;
  constexpr int TM = BM / 32, TN = BN / 32;          // 16x16 tiles per wave
  constexpr int CA = BM * BK / 8 / 256, CB = BN * BK / 8 / 256;  // 16-B chunks per thread
  __shared__ __attribute__((aligned(16))) bf16 As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1, r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  const bf16* ga[CA]; const bf16* gb[CB];
  int la[CA], lb[CB];
#pragma unroll
  for (int i = 0; i < CA; i++) {
    const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 8;
    ga[i] = X + (size_t)min(m0 + row, M - 1) * K + col;
    la[i] = row * LDK + col;
  }
#pragma unroll
  for (int i = 0; i < CB; i++) {
    const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 8;
    gb[i] = W + (size_t)min(n0 + row, N - 1) * K + col;
    lb[i] = row * LDK + col;
  }
  bf16x8 ra[CA], rbv[CB];
#pragma unroll
  for (int i = 0; i < CA; i++) ra[i] = *reinterpret_cast<const bf16x8*>(ga[i]);
#pragma unroll
  for (int i = 0; i < CB; i++) rbv[i] = *reinterpret_cast<const bf16x8*>(gb[i]);
#pragma unroll
  for (int i = 0; i < CA; i++) *reinterpret_cast<bf16x8*>(&As[0][la[i]]) = ra[i];
#pragma unroll
  for (int i = 0; i < CB; i++) *reinterpret_cast<bf16x8*>(&Bs[0][lb[i]]) = rbv[i];
  __syncthreads();

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  int cur = 0;
  for (int kt = 0; kt < nk; kt++) {
    const bool more = kt + 1 < nk;
    if (more) {
#pragma unroll
      for (int i = 0; i < CA; i++) ra[i] = *reinterpret_cast<const bf16x8*>(ga[i] + (size_t)(kt + 1) * BK);
#pragma unroll
      for (int i = 0; i < CB; i++) rbv[i] = *reinterpret_cast<const bf16x8*>(gb[i] + (size_t)(kt + 1) * BK);
    }
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
      af[i] = *reinterpret_cast<const bf16x8*>(&As[cur][(wm * (BM / 2) + i * 16 + r) * LDK + g * 8]);
#pragma unroll
    for (int j = 0; j < TN; j++)
      bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][(wn * (BN / 2) + j * 16 + r) * LDK + g * 8]);
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int i = 0; i < CA; i++) *reinterpret_cast<bf16x8*>(&As[cur ^ 1][la[i]]) = ra[i];
#pragma unroll
      for (int i = 0; i < CB; i++) *reinterpret_cast<bf16x8*>(&Bs[cur ^ 1][lb[i]]) = rbv[i];
    }
    __syncthreads();
    cur ^= 1;
  }
  const int ntiles = (N + 15) >> 4;
  epi_dispatch(ep.kind, [&](auto kc) {
    constexpr int EK = decltype(kc)::value;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int m = m0 + wm * (BM / 2) + i * 16 + 4 * g + e;
          const int n = n0 + wn * (BN / 2) + j * 16 + r;
          epi_apply<bf16, EK>(ep, m, n, acc[i][j][e], m < M && n < N, ntiles);
        }
  });
}

// ------------------------------------------------------------------------------------
// gemm_mfma2: prefill GEMM, BM x BN tile (32/64/128), BK = 64, 256 threads as 2x2 waves (wave tile
// BM/2 x BN/2), LDS double buffer fed from a PS-deep ring of register stages: the global loads of
// tile kt + PS are issued while tile kt computes (one tile of lookahead left the K loop waiting on
// HBM latency at prefill sizes, where a CU holds only 1-2 blocks).  LDS rows are 128 B (64 bf16)
// with the 16-B chunk index XOR-swizzled by (row & 7), so the 16 rows a ds_read_b128 lane group
// touches land on different chunk slots.  MFMA v_mfma_f32_16x16x32_bf16.
// ------------------------------------------------------------------------------------
// Tile order: row-major (an XCD-major remap that keeps each XCD's weight rows in its own L2 measured no
// gain: the L2 hit rate is 88 % either way at bloom-1b1 prefill sizes, profiles/r02_gemm_pmc.txt).

// Epilogue operands of one GEMM thread, loaded before the K loop (they do not depend on the sums):
// bias and int8 column scale per output column j, the residual per element, the cached positions per
// output row.  Loaded unconditionally at clamped indices: an exec-masked or per-element load in the
// epilogue makes hipcc wait for each one in turn (16-64 dependent round trips per thread).
// The residual is prefetched only for small tiles (TM * TN <= 4): a 128x128 tile's 64 values per lane would
// stay live across the whole K loop; its epilogue reads them where it uses them.
template <int TM, int TN> struct ResidPre { static constexpr bool on = TM * TN <= 4; };
template <int TM, int TN, int EK>
struct GemmEpiPre {
  float bias[TN], cscale[TN];
  float resid[EK == EPI_RESID && ResidPre<TM, TN>::on ? TM * TN * 4 : 1];
  int past[EK == EPI_QKV ? TM * 4 : 1];
};

// row_m(i, e) / col_n(j): the output row / column of accumulator element e of fragment (i, j).
template <int TM, int TN, int EK, typename RM, typename CN>
__device__ __forceinline__ void gemm_epi_prefetch(GemmEpiPre<TM, TN, EK>& pre, const Epi& ep, int M, int N, RM row_m,
                                                  CN col_n) {
  if constexpr (EK != EPI_ARGMAX) {
#pragma unroll
    for (int j = 0; j < TN; j++) {
      const int n = min(col_n(j), N - 1);
      pre.bias[j] = to_f32(((const bf16*)ep.bias)[n]);
      pre.cscale[j] = ep.col_scale ? ep.col_scale[n] : 1.f;
    }
    if constexpr (EK == EPI_RESID && ResidPre<TM, TN>::on) {
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int e = 0; e < 4; e++)
#pragma unroll
          for (int j = 0; j < TN; j++)
            pre.resid[(i * 4 + e) * TN + j] = ep.resid[(size_t)min(row_m(i, e), M - 1) * ep.ldo + min(col_n(j), N - 1)];
    }
    if constexpr (EK == EPI_QKV) {
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int e = 0; e < 4; e++)
          pre.past[i * 4 + e] = ep.past_dev ? ep.past_dev[min(row_m(i, e), M - 1) / ep.seq] : ep.past;
    }
  }
}

template <int TM, int TN, int EK, typename RM, typename CN>
__device__ __forceinline__ void gemm_epi_store(const f32x4 (&acc)[TM][TN], const GemmEpiPre<TM, TN, EK>& pre,
                                               const Epi& ep, int M, int N, RM row_m, CN col_n) {
  const int ntiles = (N + 15) >> 4;
  if constexpr (EK == EPI_ARGMAX) {
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int m = row_m(i, e), n = col_n(j);
          epi_apply<bf16, EK>(ep, m, n, acc[i][j][e], m < M && n < N, ntiles);
        }
  } else {
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int m = row_m(i, e);
#pragma unroll
        for (int j = 0; j < TN; j++) {
          const int n = col_n(j);
          if (m >= M || n >= N) continue;
          const float v = acc[i][j][e] * pre.cscale[j] + pre.bias[j];
          if constexpr (EK == EPI_QKV) {
            const int three = 3 * ep.head_dim;
            const int head = n / three, rr = n - head * three, which = rr / ep.head_dim, d = rr - which * ep.head_dim;
            if (which == 0) {
              ((bf16*)ep.q_out)[(size_t)m * ep.hidden + head * ep.head_dim + d] = from_f32<bf16>(v);
            } else {
              const int b = m / ep.seq, t = m - b * ep.seq;
              const size_t idx =
                  (((size_t)(ep.slot + b) * ep.n_head + head) * ep.max_ctx + pre.past[i * 4 + e] + t) * ep.head_dim + d;
              ((bf16*)(which == 1 ? ep.k_cache : ep.v_cache))[idx] = from_f32<bf16>(v);
            }
          } else if constexpr (EK == EPI_RESID) {
            const float rs = ResidPre<TM, TN>::on ? pre.resid[(i * 4 + e) * TN + j] : ep.resid[(size_t)m * ep.ldo + n];
            ep.out_f32[(size_t)m * ep.ldo + n] = v + rs;
          } else {
            ((bf16*)ep.out_act)[(size_t)m * ep.ldo + n] = from_f32<bf16>(gelu_bloom(v));
          }
        }
      }
  }
}

// Split-K (gridDim.z = KS > 1, K % (KS * 64) == 0): block z computes columns [z K / KS, (z + 1) K / KS) of
// the dot products, stores its partial tile write-through (sc1) to ep.sk_ws in fragment order
// ([tile][z][wave][i][j][lane] f32x4: 16 B per lane, coalesced) and takes the tile's ticket; the block
// drawing the last ticket sums the KS partials in z order (its own from registers: the same order
// whichever block arrives last, so results do not depend on timing), resets the ticket and runs the
// epilogue.  MI355X_MICROARCH.md "Valid forms" row 1 (counter form, the last adder reads).
template <int BM, int BN, int PS, int EK>
__global__ __launch_bounds__(256) void gemm_mfma2_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                         int M, int N, int K, Epi ep) {
  constexpr int BK = 64;
  constexpr int TM = BM / 32, TN = BN / 32;           // 16x16 tiles per wave (wave = BM/2 x BN/2)
  constexpr int CA = BM * BK / 8 / 256, CB = BN * BK / 8 / 256;  // 16-B chunks per thread: 4, 4|2|1
  __shared__ __attribute__((aligned(16))) bf16 As[2][BM * BK];
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][BN * BK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1, r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int KS = gridDim.z, kz = blockIdx.z, Kz = K / KS;  // this block's K range: [kz Kz, (kz + 1) Kz)
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); };  // element offset
  auto row_m = [&](int i, int e) { return m0 + wm * (BM / 2) + i * 16 + 4 * g + e; };
  auto col_n = [&](int j) { return n0 + wn * (BN / 2) + j * 16 + r; };

  GemmEpiPre<TM, TN, EK> pre;
  gemm_epi_prefetch(pre, ep, M, N, row_m, col_n);

  const bf16* ga[CA]; const bf16* gb[CB];
  int la[CA], lb[CB];
#pragma unroll
  for (int i = 0; i < CA; i++) {
    const int c = tid + i * 256, row = c >> 3, ch = c & 7;
    ga[i] = X + (size_t)min(m0 + row, M - 1) * K + (size_t)kz * Kz + ch * 8;
    la[i] = sw(row, ch);
  }
#pragma unroll
  for (int i = 0; i < CB; i++) {
    const int c = tid + i * 256, row = c >> 3, ch = c & 7;
    gb[i] = W + (size_t)min(n0 + row, N - 1) * K + (size_t)kz * Kz + ch * 8;
    lb[i] = sw(row, ch);
  }
  const int nk = Kz / BK;
  bf16x8 ra[PS][CA], rb[PS][CB];
  auto gload = [&](int st, int kt) {  // tile kt -> register stage st (clamped: a re-read past the end is unused)
    const size_t off = (size_t)min(kt, nk - 1) * BK;
#pragma unroll
    for (int i = 0; i < CA; i++) ra[st][i] = *reinterpret_cast<const bf16x8*>(ga[i] + off);
#pragma unroll
    for (int i = 0; i < CB; i++) rb[st][i] = *reinterpret_cast<const bf16x8*>(gb[i] + off);
  };
  auto lstore = [&](int st, int buf) {
#pragma unroll
    for (int i = 0; i < CA; i++) *reinterpret_cast<bf16x8*>(&As[buf][la[i]]) = ra[st][i];
#pragma unroll
    for (int i = 0; i < CB; i++) *reinterpret_cast<bf16x8*>(&Bs[buf][lb[i]]) = rb[st][i];
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto ktile = [&](int buf) {  // the MFMAs of one BK-deep tile from LDS buffer buf
#pragma unroll
    for (int ks = 0; ks < BK / 32; ks++) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; i++)
        af[i] = *reinterpret_cast<const bf16x8*>(&As[buf][sw(wm * (BM / 2) + i * 16 + r, ks * 4 + g)]);
#pragma unroll
      for (int j = 0; j < TN; j++)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[buf][sw(wn * (BN / 2) + j * 16 + r, ks * 4 + g)]);
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // Ring: tiles 0..PS-1 in flight, tile 0 -> LDS, stage 0 refilled with tile PS.  Step kt computes
  // LDS buffer cur, stores tile kt + 1 (register stage (kt + 1) % PS) into the other buffer and
  // refills that stage with tile kt + 1 + PS.  Full groups of PS steps run with no conditions at all
  // (loads past the end re-read the last tile; a store past the end fills a buffer nobody reads), so
  // the compiler counts the ring's loads with vmcnt(N) instead of draining them every step.
#pragma unroll
  for (int st = 0; st < PS; st++) gload(st, st);
  lstore(0, 0);
  gload(0, PS);
  __syncthreads();
  int cur = 0, kt0 = 0;
  for (; kt0 + PS <= nk; kt0 += PS) {
#pragma unroll
    for (int s2 = 0; s2 < PS; s2++) {
      const int kt = kt0 + s2, nst = (s2 + 1) % PS;
      ktile(cur);
      lstore(nst, cur ^ 1);
      gload(nst, kt + 1 + PS);
      __syncthreads();
      cur ^= 1;
    }
  }
#pragma unroll
  for (int s2 = 0; s2 < PS; s2++) {  // tail: nk % PS steps
    const int kt = kt0 + s2, nst = (s2 + 1) % PS;
    if (kt < nk) {
      ktile(cur);
      lstore(nst, cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }
  if (KS > 1) {
    __shared__ int last;
    const size_t tile = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    float* base = ep.sk_ws + tile * KS * (BM * BN);
    const __amdgpu_buffer_rsrc_t rs = attn_rsrc(base);
    auto off = [&](int z, int i, int j) { return (uint32_t)(((((z * 4 + w) * TM + i) * TN + j) * 64 + lane) * 16); };
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[i][j]), rs, off(kz, i, j), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      typedef __attribute__((address_space(1))) unsigned gu32;
      const unsigned old = __hip_atomic_fetch_add((gu32*)(ep.sk_tickets + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == (unsigned)(KS - 1);
      if (last) __hip_atomic_store((gu32*)(ep.sk_tickets + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++) {
        f32x4 t = (f32x4){0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < KS; z++)
          t += z == kz ? acc[i][j] : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off(z, i, j), 0, 16));
        acc[i][j] = t;
      }
  }
  gemm_epi_store(acc, pre, ep, M, N, row_m, col_n);
}

// ------------------------------------------------------------------------------------
// gemm_mfma3: prefill GEMM on v_mfma_f32_32x32x16_bf16 (measured 2184 TFLOP/s against 1272 for the 16x16x32
// form, bs_mfma_probe).  128 x 128 tile, 512 threads as 2 x 4 waves of 64 x 32 (two 32 x 32 accumulators;
// two waves per SIMD, so one's MFMAs run while the other waits on LDS), BK = 64.  Staging is LDS-DMA
// (buffer_load ... lds: no VGPR round trip, no ds_write pass) into 3 LDS stages (96 KB): tile kt computes
// while tiles kt + 1 and kt + 2 land, one raw s_barrier per step.
// Stream-K work split: at prefill sizes the tile count is small and uneven against 256 CUs (bloom-1b1 QKV
// at 512 tokens: 144 tiles x 24 K-steps), so the tiles x K-steps iteration space is cut into gridDim.x equal
// contiguous ranges, one per block.  A block runs the tile segments its range covers; a whole tile goes
// straight to the epilogue, a partial one stores its fp32 fragments (write-through, slab 2 b + 0 for the
// block's first segment, 2 b + 1 for its last) and takes the tile's ticket; the block drawing the last
// ticket sums the tile's segments in K order (whichever block arrives last: deterministic) and runs the
// epilogue (LDS-staged: 16-B stores).  Per block (tools/gemm3_stamps.hip, profiles/r03_gemm3_stamps*.txt):
// ~0.52 us per 64-deep K-step, ~0.8 us prologue, ~2.5-3.5 us epilogue.
// Fragment maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) holds A[row r][k 8h + j]
// = X[m][k] and B[k 8h + j][col r] = W[n][k]; accumulator register e is row (e & 3) + 8 (e >> 2) + 4 h,
// column r.  LDS rows are 128 B with the 16-B chunk index XOR-swizzled by (row >> 1) & 7: the 16 lanes
// of a ds_read_b128 pass (rows 2k, 2k + 1 in the two halves of a 256-B bank row) hit 16 distinct slots.
// ------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
#ifdef GEMM3_STAMPS
__device__ unsigned long long g_gemm3_stamps[4096 * 4];
#endif

// Stream-K geometry shared by the kernel and the host: block bb's first iteration, and the block owning
// iteration x (the largest bb with first(bb) <= x).
__host__ __device__ __forceinline__ long gemm3_first(int bb, long T, int G) { return (long)bb * T / G; }
__host__ __device__ __forceinline__ int gemm3_owner(long x, long T, int G) { return (int)(((x + 1) * G + T - 1) / T - 1); }

// XCD-aware placement (XM): workgroups are dispatched round-robin over the 8 XCDs (block i on XCD i % 8), each
// XCD with its own 4 MB L2.  Virtual block v = (i % 8) * (G / 8) + i / 8 gives every XCD one contiguous eighth
// of the iteration space, and tiles are numbered column-major (all M tiles of a W column tile in a row), so an
// XCD streams ~1/8 of W (+ all of X) instead of every XCD streaming all of W from the Infinity Cache.
__host__ __device__ __forceinline__ int gemm3_vblock(int i, int G) { return G % 8 ? i : (i % 8) * (G / 8) + i / 8; }

// NSTG LDS stages: 3 (one block per CU) or 2 (two per CU at BN = 128).  BN_ = 128: 8 waves of 64 x 32; BN_ = 256
// (wide tiles for wide N: bloom-7b1's QKV / fc1 at 512 tokens are 192 / 256 whole 128 x 256 tiles, one per CU, no
// partial tiles, a third less staging per MFMA): 8 waves of 64 x 64, 144 KB of LDS.
// BM_ = 256 (with BN_ = 256, round 6): 256 x 256 tiles for the large prefills (configs[4]'s 16 rows x up to 2048 tokens),
// 8 waves of 128 x 64 -- half the LDS fragment reads per MFMA of the 128-row tiles; two LDS stages (128 KB), the
// epilogue staged in four 64-row passes.
template <int EK, int NSTG = 3, bool XM = true, int BN_ = 128, int BM_ = 128>
__global__ __launch_bounds__(512) void gemm_mfma3_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                         int M, int N, int K, Epi ep) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass dropped this template's launch stubs (no diagnostic) without it
  constexpr int BM = BM_, BN = BN_, BK = 64;
  static_assert(BM == 128 || (BM == 256 && BN == 256), "256-row tiles come with 256 columns");
  constexpr int FI = BM / 64;  // 32-row fragments per wave (the wave's rows: BM / 2)
  // waves: 2 (M) x WN (N) of 64 x WNC; BN = 128: 8 waves of 64 x 32 (2 per SIMD, one's MFMAs cover the other's LDS
  // waits); BN = 256: 8 waves of 64 x 64; BN = 96: 6 waves of 64 x 32 (two-thirds of the 128 x 128 block's
  // staging and fragment reads per step for three-quarters of its MFMAs: more whole tiles where 128 x 128 leaves
  // CUs idle)
  constexpr int WN = BN == 256 ? 4 : BN / 32;
  constexpr int FJ = BN == 256 ? 2 : 1, WNC = BN / WN;  // 32-column fragments per wave, columns per wave
  constexpr int NTH = 128 * WN;
  // 16-B chunks per thread per stage (A rounded up to whole wave instructions: the LDS A region is padded so the
  // extra DMAs land in slots nobody reads, and every wave counts the same DMAs per stage)
  constexpr int CA = (BM * BK / 8 + NTH - 1) / NTH, CB = BN * BK / 8 / NTH;
  constexpr int APAD = CA * NTH * 8;             // bf16 elements of a stage's A region
  constexpr int SLD = BN + 8;                    // epilogue staging row stride (floats)
  // epilogue rows staged per pass: the whole 128-row tile at once; 64 rows at a time for 256-row tiles (the wave's 128
  // accumulators stay live until its pass, so a pass's residual prefetch must stay small: 128-row passes spilled)
  constexpr int EPR = BM == 128 ? 128 : 64, NPASS = BM / EPR;
  constexpr int SMEM = NSTG * (APAD + BN * BK) > EPR * SLD * 2 ? NSTG * (APAD + BN * BK) : EPR * SLD * 2;  // + staging
  __shared__ __attribute__((aligned(16))) bf16 smem[SMEM];  // 96 KB at 3 stages of 128 x 128, the only LDS object
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w - wm * WN, r = lane & 31, h = lane >> 5;  // wave tile 64 x WNC at (64 wm, WNC wn)
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM, nk = K / BK;
  const long T = (long)tiles_n * tiles_m * nk;
  const int G = gridDim.x, b = XM ? gemm3_vblock(blockIdx.x, G) : blockIdx.x;
  const long it_begin = gemm3_first(b, T, G), it_end = gemm3_first(b + 1, T, G);
#ifdef GEMM3_STAMPS
  const unsigned long long st0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st1 = 0, st2 = 0;
#endif
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); };
  auto As = [&](int buf) { return smem + buf * (APAD + BN * BK); };
  auto Bs = [&](int buf) { return smem + buf * (APAD + BN * BK) + APAD; };
  // Staging: buffer loads straight into LDS (LDS-DMA, no VGPR round trip), a 32-bit byte offset per lane
  // and the K position as the scalar offset (the host checks M * K and N * K bf16 fit 4 GB).  An LDS-DMA
  // instruction writes 64 consecutive 16-B slots (wave-uniform base + 16 lane), so the XOR swizzle is
  // applied on the global side: the lane filling slot s of row `row` fetches logical chunk s ^ f(row).
  // operand descriptors bounded to the operands (the host checks they fit 4 GB): an offset past them reads 0
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(X), (short)0,
                                                                       (int)(uint32_t)((size_t)M * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(W), (short)0,
                                                                       (int)(uint32_t)((size_t)N * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = attn_rsrc(ep.sk_ws);
  auto slab_off = [&](int slab, int i, int j, int q) {
    return (uint32_t)(((((((size_t)slab * 8 + w) * FI + i) * FJ + j) * 4 + q) * 64 + lane) * 16);
  };
  int* flag = reinterpret_cast<int*>(smem);
  f32x16 acc[FI][FJ];

  for (long it = it_begin; it < it_end;) {
    const int t = (int)(it / nk), k0 = (int)(it - (long)t * nk);
    const int kn = (int)min((long)(nk - k0), it_end - it);  // K-steps of this segment
    const int tn = XM ? t / tiles_m : t - (t / tiles_n) * tiles_n, tm = XM ? t - tn * tiles_m : t / tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const bool first_seg = it == it_begin;
    it += kn;
    uint32_t oa[CA], ob[CB];  // CB = 2 CA at BN = 256: A and B offsets in separate loops
#pragma unroll
    for (int i = 0; i < CA; i++) {
      const int c = i * NTH + w * 64 + lane, row = c >> 3, ch = (c & 7) ^ ((row >> 1) & 7);
      oa[i] = (uint32_t)(((size_t)min(m0 + row, M - 1) * K + (size_t)k0 * BK + ch * 8) * 2);
    }
#pragma unroll
    for (int i = 0; i < CB; i++) {
      const int c = i * NTH + w * 64 + lane, row = c >> 3, ch = (c & 7) ^ ((row >> 1) & 7);
      ob[i] = (uint32_t)(((size_t)min(n0 + row, N - 1) * K + (size_t)k0 * BK + ch * 8) * 2);
    }
    static_assert(CA * NTH * 8 >= BM * BK && CB * NTH * 8 == BN * BK, "every staged chunk has one lane");
    float bias[FJ], cscale[FJ];
#pragma unroll
    for (int j = 0; j < FJ; j++) {
      const int n = min(n0 + wn * WNC + j * 32 + r, N - 1);
      bias[j] = to_f32(((const bf16*)ep.bias)[n]);
      cscale[j] = ep.col_scale ? ep.col_scale[n] : 1.f;
    }
    typedef __attribute__((address_space(3))) void lds_void;
    auto gload = [&](int buf, int kt) {  // segment step kt -> LDS stage buf (clamped: a re-load past the end is unread)
      const int off = min(kt, kn - 1) * BK * 2;
#pragma unroll
      for (int i = 0; i < CA; i++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)(As(buf) + (i * NTH + w * 64) * 8), 16, oa[i], off, 0, 0);
#pragma unroll
      for (int i = 0; i < CB; i++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(Bs(buf) + (i * NTH + w * 64) * 8), 16, ob[i], off, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < FI; i++)
#pragma unroll
      for (int j = 0; j < FJ; j++)
#pragma unroll
        for (int e = 0; e < 16; e++) acc[i][j][e] = 0.f;
    auto ktile = [&](int buf) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ks++) {
        bf16x8 af[FI], bfr[FJ];
#pragma unroll
        for (int i = 0; i < FI; i++) af[i] = *reinterpret_cast<const bf16x8*>(As(buf) + sw(wm * (BM / 2) + i * 32 + r, ks * 2 + h));
#pragma unroll
        for (int j = 0; j < FJ; j++) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs(buf) + sw(wn * WNC + j * 32 + r, ks * 2 + h));
#pragma unroll
        for (int i = 0; i < FI; i++)
#pragma unroll
          for (int j = 0; j < FJ; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    // Step kt: this wave's DMA of tile kt retired (vmcnt(CA + CB) leaves tile kt + 1's in flight) ->
    // barrier (every wave's part of tile kt has landed; every wave is done reading tile kt - 1) -> DMA of
    // tile kt + 2 into tile kt - 1's stage -> MFMAs of tile kt.  One barrier per step, raw s_barrier: a
    // __syncthreads() would also wait vmcnt(0) and drain the DMA in flight (cdna_hip_programming.md §5,
    // "Pipelining across barriers").  The previous segment's epilogue ended with a barrier: the LDS is free.
    gload(0, 0);
    if constexpr (NSTG == 3) gload(1, 1);
#ifdef GEMM3_STAMPS
    if (first_seg) st1 = __builtin_amdgcn_s_memrealtime();
#endif
    int buf = 0, nbuf = NSTG - 1;  // stage of tile kt, stage for tile kt + NSTG - 1
    for (int kt = 0; kt < kn; kt++) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + CB)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      gload(nbuf, kt + NSTG - 1);
      ktile(buf);
      buf = buf == NSTG - 1 ? 0 : buf + 1;
      nbuf = nbuf == NSTG - 1 ? 0 : nbuf + 1;
    }
    // the clamped DMAs past the end land before the LDS is reused (partials' flag, epilogue staging)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#ifdef GEMM3_STAMPS
    if (first_seg) st2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (kn < nk) {
      // partial tile: fragments out, ticket; the last arriver sums the tile's segments in K order
      const int slab = 2 * b + (first_seg ? 0 : 1);
#pragma unroll
      for (int i = 0; i < FI; i++)
#pragma unroll
        for (int j = 0; j < FJ; j++)
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), rs, slab_off(slab, i, j, q), 0, 16);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int b_first = gemm3_owner((long)t * nk, T, G), b_last = gemm3_owner((long)(t + 1) * nk - 1, T, G);
      __syncthreads();
      if (tid == 0) {
        typedef __attribute__((address_space(1))) unsigned gu32;
        const unsigned old = __hip_atomic_fetch_add((gu32*)(ep.sk_tickets + t), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(b_last - b_first);
        if (last) __hip_atomic_store((gu32*)(ep.sk_tickets + t), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      const int is_last = *flag;
      __syncthreads();  // the flag word is LDS the next segment overwrites
      if (!is_last) continue;
#pragma unroll
      for (int i = 0; i < FI; i++)
#pragma unroll
        for (int j = 0; j < FJ; j++) {
          f32x4 sum[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
          for (int bb = b_first; bb <= b_last; bb++) {
            const int sl = 2 * bb + (gemm3_first(bb, T, G) >= (long)t * nk ? 0 : 1);
            f32x4 v[4];
#pragma unroll
            for (int q = 0; q < 4; q++) v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, slab_off(sl, i, j, q), 0, 16));
#pragma unroll
            for (int q = 0; q < 4; q++) sum[q] += v[q];
          }
#pragma unroll
          for (int q = 0; q < 4; q++)
#pragma unroll
            for (int e = 0; e < 4; e++) acc[i][j][4 * q + e] = sum[q][e];
        }
    }
    // Epilogue through LDS (the staging buffers are dead): the whole tile is written there as fp32 (acc *
    // col_scale + bias; row stride BN + 8 floats, so the two lane halves of a store hit disjoint banks; 68 KB of
    // the 96 KB at BN = 128), one barrier, then read back as 8-column chunks: one 16-B bf16 store (GELU, QKV) or two 16-B fp32
    // loads + stores (RESID) per chunk instead of 64 per-element accesses per lane.  The residual chunks and the
    // rows' cached lengths are loaded before the staging (clamped, unconditional: one round trip).
    constexpr int NCH = EPR * BN / 8 / NTH, CPR = BN / 8;  // chunks per thread per pass (4 or 8), chunks per row
    float* stg = reinterpret_cast<float*>(smem);
    auto chunk_rc = [&](int c, int& lr, int& lc) { const int id = tid + c * NTH; lr = id / CPR; lc = (id % CPR) * 8; };
#pragma unroll
    for (int pass = 0; pass < NPASS; pass++) {
      const int r0 = pass * EPR;  // the pass's first row of the tile (BM = 256: the rows of waves wm == pass)
      f32x4 rsd[NCH][2];
      int cpast[NCH];
      auto epi_loads = [&]() {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
          int lr, lc;
          chunk_rc(c, lr, lc);
          const int m = min(m0 + r0 + lr, M - 1), n = min(n0 + lc, N - 8);
          if constexpr (EK == EPI_RESID) {
            rsd[c][0] = *reinterpret_cast<const f32x4*>(ep.resid + (size_t)m * ep.ldo + n);
            rsd[c][1] = *reinterpret_cast<const f32x4*>(ep.resid + (size_t)m * ep.ldo + n + 4);
          }
          if constexpr (EK == EPI_QKV) cpast[c] = ep.past_dev ? ep.past_dev[m / ep.seq] : ep.past;
        }
      };
      epi_loads();  // the residual / position loads go out before the staging (one round trip under it)
#pragma unroll
      for (int i = 0; i < FI; i++) {
        if (NPASS > 1 && (wm * (BM / 2) + i * 32) / EPR != pass) continue;  // wave-uniform: fragment i is another pass's
#pragma unroll
        for (int j = 0; j < FJ; j++)
#pragma unroll
          for (int e = 0; e < 16; e++)
            stg[(wm * (BM / 2) - r0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * SLD + wn * WNC + j * 32 + r] =
                acc[i][j][e] * cscale[j] + bias[j];
      }
      __syncthreads();
#pragma unroll
      for (int c = 0; c < NCH; c++) {
        int lr, lc;
        chunk_rc(c, lr, lc);
        const int m = m0 + r0 + lr, n = n0 + lc;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(stg + lr * SLD + lc);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(stg + lr * SLD + lc + 4);
        if (m >= M || n >= N) continue;
        if constexpr (EK == EPI_RESID) {
          float* o = ep.out_f32 + (size_t)m * ep.ldo + n;
          *reinterpret_cast<f32x4*>(o) = v0 + rsd[c][0];
          *reinterpret_cast<f32x4*>(o + 4) = v1 + rsd[c][1];
        } else {
          bf16x8 b8;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            b8[q] = from_f32<bf16>(EK == EPI_GELU ? gelu_bloom(v0[q]) : v0[q]);
            b8[4 + q] = from_f32<bf16>(EK == EPI_GELU ? gelu_bloom(v1[q]) : v1[q]);
          }
          if constexpr (EK == EPI_GELU) {
            *reinterpret_cast<bf16x8*>((bf16*)ep.out_act + (size_t)m * ep.ldo + n) = b8;
          } else {
            const int three = 3 * ep.head_dim;
            const int head = n / three, rr = n - head * three, which = rr / ep.head_dim, d = rr - which * ep.head_dim;
            bf16* dst;
            if (which == 0) {
              dst = (bf16*)ep.q_out + (size_t)m * ep.hidden + head * ep.head_dim + d;
            } else {
              const int bi = m / ep.seq, ti = m - bi * ep.seq;
              dst = (bf16*)(which == 1 ? ep.k_cache : ep.v_cache) +
                    (((size_t)(ep.slot + bi) * ep.n_head + head) * ep.max_ctx + cpast[c] + ti) * ep.head_dim + d;
            }
            *reinterpret_cast<bf16x8*>(dst) = b8;
          }
        }
      }
      if (NPASS > 1 && pass + 1 < NPASS) __syncthreads();  // the staging rows are rewritten by the next pass
    }
    __syncthreads();  // the staging rows are overwritten next (the next segment's tiles)
  }
#ifdef GEMM3_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long st3 = __builtin_amdgcn_s_memrealtime();
  if (tid < 4 && b < 4096) g_gemm3_stamps[b * 4 + tid] = tid == 0 ? st0 : tid == 1 ? st1 : tid == 2 ? st2 : st3;
#endif
#endif
}

// Grid of gemm_mfma3 (0: use another kernel), from the per-block costs tools/gemm3_stamps.hip measured
// (~0.8 us prologue, ~2.5-3.5 us epilogue, ~0.52 us per 64-deep K-step at one block per CU) and the sweeps
// against gemm_mfma2 (profiles/r03_gemm3.txt): 256 blocks (one per CU, stream-K ranges over the tiles) when
// there are >= 256 tiles; otherwise tiles x KS blocks with KS = 256 / tiles (at most 4) splitting K, taken only
// when a block keeps >= 16 K-steps (short-K narrow shapes like bloom-1b1's dense stay on 64 x 64 tiles).
// Conditions: K % 64 == 0, N % 8 == 0, QKV head_dim % 8 == 0, operands under 4 GB (32-bit buffer offsets),
// partial slabs (2 per block, 64 KB each) in the workspace, one ticket per tile.
static int gemm3_grid(int M, int N, int K, const Epi& ep) {
  if (K % 64 || N % 8 || ep.kind == EPI_ARGMAX) return 0;
  if (ep.kind == EPI_QKV && ep.head_dim % 8) return 0;
  if ((size_t)M * K * 2 >= (1ull << 32) || (size_t)N * K * 2 >= (1ull << 32)) return 0;
  if (!ep.sk_ws || !ep.sk_tickets) return 0;
  const long tiles = (long)((M + 127) / 128) * ((N + 127) / 128);
  const long nk = K / 64;
  long G;
  if (tiles >= 256) {
    G = 256;
  } else {
    const long ks = std::max(1L, std::min(4L, 256 / tiles));
    if (nk / ks < 16) return 0;
    G = tiles * ks;
  }
  if (tiles > ep.sk_ntickets || (size_t)2 * G * 128 * 128 > ep.sk_cap) return 0;
  return (int)G;
}

// Wide tiles (BN = 256): whole 128 x 256 tiles, one per block, when they fill 160..256 CUs with >= 32 K-steps each
// (bloom-7b1 QKV / fc1 at 512 tokens: 192 / 256 tiles, where 128 x 128 tiles are 384 / 512 and stream-K splits
// half of them; hipBLASLt picks one-tile-per-CU grids of wide tiles there too, profiles/r04_hipblaslt_kernels.txt).
// G = tiles: every block's stream-K range is exactly one tile's K loop, so no partial tile, slab or ticket.
static int gemm3_wide_grid(int M, int N, int K, const Epi& ep) {
  if (K % 64 || N % 256 || ep.kind == EPI_ARGMAX) return 0;
  if (ep.kind == EPI_QKV && ep.head_dim % 8) return 0;
  if ((size_t)M * K * 2 >= (1ull << 32) || (size_t)N * K * 2 >= (1ull << 32)) return 0;
  const long tiles = (long)((M + 127) / 128) * (N / 256);
  if (tiles < 160 || tiles > 256 || K / 64 < 32) return 0;
  return (int)tiles;
}

// Two blocks per CU (2 LDS stages, 68 KB each) on whole tiles: when the 128 x 128 tiles number >= 384 and split
// evenly over 512 (or 384) blocks, every block runs whole tiles (no partial tile) and a second block per CU
// covers the first one's barriers and epilogue: bloom-7b1 QKV at 2048 tokens 257 -> 233 us, fc1 at 1024 tokens
// 175 -> 154 us, bloom-1b1 QKV at 4096 tokens (1152 tiles, 384 blocks) 109 -> 98 us
// (profiles/r04_gemm_long_prompts.txt).
static int gemm3_pair_grid(int M, int N, int K, const Epi& ep) {
  if (K % 64 || N % 8 || ep.kind == EPI_ARGMAX || K / 64 < 16) return 0;
  if (ep.kind == EPI_QKV && ep.head_dim % 8) return 0;
  if ((size_t)M * K * 2 >= (1ull << 32) || (size_t)N * K * 2 >= (1ull << 32)) return 0;
  const long tiles = (long)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles < 384) return 0;
  if (tiles % 512 == 0) return 512;
  if (tiles % 384 == 0) return 384;  // 384 tiles: one per block (bloom-1b1 fc1 at 1024 tokens 38.0 -> 31.5 us)
  return 0;
}

template <int NSTG = 3, bool XM = true, int BN = 128, int BM = 128>
static void gemm3_launch(const bf16* x, const bf16* w, int M, int N, int K, const Epi& ep, hipStream_t s, int G) {
  constexpr int NTH = BN == 256 ? 512 : 128 * (BN / 32);
  switch (ep.kind) {
    case EPI_QKV: gemm_mfma3_kernel<EPI_QKV, NSTG, XM, BN, BM><<<G, NTH, 0, s>>>(x, w, M, N, K, ep); break;
    case EPI_RESID: gemm_mfma3_kernel<EPI_RESID, NSTG, XM, BN, BM><<<G, NTH, 0, s>>>(x, w, M, N, K, ep); break;
    default: gemm_mfma3_kernel<EPI_GELU, NSTG, XM, BN, BM><<<G, NTH, 0, s>>>(x, w, M, N, K, ep); break;
  }
}

// 256 x 256 tiles (round 6): one whole tile per block (G = tiles: no partial tile, slab or ticket), two LDS stages,
// for the big prefills (>= 16 K-steps, K <= 8192: bloom-7b1 fc2's K = 16384 ran 0.90-0.95x).  bloom-7b1 QKV at 4096
// tokens 645 -> 397 us (639 -> 1040 TFLOP/s), fc1 605 -> 553, dense 164 -> 147; bloom-3b QKV 246 -> 185; every output
// bit-identical to the 128 x 128 path (same K order).  0: not applicable.
static int gemm3_big_grid(int M, int N, int K, const Epi& ep) {
  // BS_GEMM_BIG=0 turns the 256 x 256 tiles off (tests compare the two paths bit for bit); read per call: prefill only
  const char* off = getenv("BS_GEMM_BIG");
  if (off && off[0] == '0') return 0;
  if (K % 64 || N % 8 || ep.kind == EPI_ARGMAX || K / 64 < 16 || K > 8192) return 0;
  if (ep.kind == EPI_QKV && ep.head_dim % 8) return 0;
  if ((size_t)M * K * 2 >= (1ull << 32) || (size_t)N * K * 2 >= (1ull << 32)) return 0;
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  // >= 256 tiles that fill their last round of blocks to >= 70 % (288 tiles leave 224 CUs idle in the second round:
  // bloom-1b1 QKV at 4096 tokens 0.96x; 256 / 384 / 480 tiles 1.12-1.33x, profiles/r06_gemm_256x256_ab.txt)
  const long rounds = (tiles + 255) / 256;
  if (tiles < 256 || tiles * 10 < rounds * 256 * 7 || tiles > (1L << 20)) return 0;
  return (int)tiles;
}

// 128 x 96 tiles (6 waves), whole tiles, one per block: where 128 x 128 tiles leave CUs idle (< 200 tiles) and the
// 128 x 96 grid fills 160..256 CUs with 16..40 K-steps per tile (tools/gemm_splitk_bench.hip, profiles/r05_gemm_n96.txt:
// bloom-1b1 QKV at 512 tokens 144 tiles of 128 x 128 -> 192 of 128 x 96, 18.8 -> 17.3 us; fc1 20.1 -> 19.7; bloom-3b
// dense at 1024 tokens 26.7 -> 25.6; long K loses: bloom-7b1 fc2 91 -> 112).  0: not applicable.
static int gemm3_n96_grid(int M, int N, int K, const Epi& ep) {
  if (K % 64 || N % 8 || ep.kind == EPI_ARGMAX || K / 64 < 16 || K / 64 > 40) return 0;
  if (ep.kind == EPI_QKV && ep.head_dim % 8) return 0;
  if ((size_t)M * K * 2 >= (1ull << 32) || (size_t)N * K * 2 >= (1ull << 32)) return 0;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  const long t96 = (long)((M + 127) / 128) * ((N + 95) / 96);
  if (t128 >= 200 || t96 < 160 || t96 > 256) return 0;
  return (int)t96;
}

// gemm_mfma2_kernel with the epilogue kind as a template argument.
template <int BM, int BN, int PS>
static void gemm2_launch(const bf16* x, const bf16* w, int M, int N, int K, const Epi& ep, hipStream_t s, int KS = 1) {
  const dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, KS);
  switch (ep.kind) {
    case EPI_QKV: gemm_mfma2_kernel<BM, BN, PS, EPI_QKV><<<grid, 256, 0, s>>>(x, w, M, N, K, ep); break;
    case EPI_RESID: gemm_mfma2_kernel<BM, BN, PS, EPI_RESID><<<grid, 256, 0, s>>>(x, w, M, N, K, ep); break;
    case EPI_GELU: gemm_mfma2_kernel<BM, BN, PS, EPI_GELU><<<grid, 256, 0, s>>>(x, w, M, N, K, ep); break;
    default: gemm_mfma2_kernel<BM, BN, PS, EPI_ARGMAX><<<grid, 256, 0, s>>>(x, w, M, N, K, ep); break;
  }
}

// ------------------------------------------------------------------------------------
// gemm_f32: exact-fp32 path (parity mode).  16x16 output tile per 256-thread block.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                       int M, int N, int K, Epi ep) {
  __shared__ float Xs[16][17], Ws[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
  float acc = 0.f;
  const float* xr = X + (size_t)min(m0 + ty, M - 1) * K;
  const float* wr = W + (size_t)min(n0 + ty, N - 1) * K;
  for (int k0 = 0; k0 < K; k0 += 16) {
    Xs[ty][tx] = xr[k0 + tx];
    Ws[ty][tx] = wr[k0 + tx];
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk++) acc += Xs[ty][kk] * Ws[tx][kk];
    __syncthreads();
  }
  const int m = m0 + ty, n = n0 + tx;
  epi_dispatch(ep.kind, [&](auto kc) {
    epi_apply<float, decltype(kc)::value>(ep, m, n, acc, m < M && n < N, (N + 15) >> 4);
  });
}

template <int WAVES, int MT, bool LN>
static void gemv_launch(const bf16* X, const LnArgs& ln, const bf16* W, int M, int N, int K, const Epi& ep,
                        hipStream_t s) {
  size_t shm = sizeof(float) * WAVES * MT * 16 * 17;
  if (LN) shm += (size_t)M * K * sizeof(bf16);
  // U = 4, plain (not non-temporal) loads, no software prefetch: the fastest variant in the
  // tools/gemv_bench.hip A/B (profiles/r01_gemv_bench.log)
  gemv_mfma_kernel<WAVES, MT, 4, LN, 0, 0><<<(N + 15) / 16, WAVES * 64, shm, s>>>(W, X, ln, M, N, K, ep);
}

static int gemv_waves(int N, int K) {
  const int ntiles = (N + 15) / 16, ksteps = K / 32;
  int waves = 4;
  while (waves < 16 && ntiles * waves < 2048 && waves * 2 <= ksteps) waves *= 2;
  return waves;
}

template <int R, int MM, int XM, int U = 2, int FL = 0>
static void gemv_rows_launch(const bf16* X, const LnArgs& ln, const AttnParts& pa, const bf16* W, int M, int N,
                             int K, const Epi& ep, hipStream_t s, int waves = 4) {
  const size_t shm = 256 + (XM != X_PLAIN ? (size_t)M * K * sizeof(bf16) : 0);
  const int blocks = (N + waves * R - 1) / (waves * R);
  if (waves <= 4) {
    gemv_rows_kernel<R, MM, U, XM, FL, 256><<<blocks, waves * 64, shm, s>>>(W, X, ln, pa, M, N, K, ep);
  } else if constexpr (MM <= 2) {  // wide blocks: <= 128 VGPRs (rows_geometry keeps R x U small)
    gemv_rows_kernel<R, MM, U, XM, FL, 1024><<<blocks, waves * 64, shm, s>>>(W, X, ln, pa, M, N, K, ep);
  }
}

// Rows GEMV geometry: every CU streams the same number of weight bytes.  A CU pulls ~24 GB/s of a
// chip-wide stream (MI355X_MICROARCH.md: ~10 B/cycle/CU), so a grid of 4-wave blocks that puts 3 blocks
// on some CUs and 2 on others (bloom-1b1 QKV: 576 blocks) ends when the 3-block CUs do: the in-kernel
// timeline (tools/gemv_timeline.hip) showed 2 us between the first and last block's end.  Here a block
// holds ceil(N / 256) rows (R per wave, <= 16 waves), so the grid is ~256 equal blocks.
static void rows_geometry(int N, int K, int M, int r_default, int* R, int* waves) {
  if (M > 2) { *R = r_default; *waves = 4; return; }
  const int rows_cu = (N + 255) / 256;
  int r = K <= 2048 ? 2 : 1;
  while ((rows_cu + r - 1) / r > 16 && r < 4) r *= 2;
  if ((rows_cu + r - 1) / r < 4) r = 1;  // the LayerNorm / merge prologues need >= 4 waves (256 threads)
  *R = r;
  *waves = std::max(4, std::min(16, (rows_cu + r - 1) / r));
}

// Geometry of a non-argmax rows GEMV: rows per wave R, waves per block, 512-column chunks in flight U.
static void rows_plan(int XM, int M, int N, int K, int* R, int* waves, int* U) {
  const bool LN = XM == X_LN || XM == X_EMB;
  // rows per wave (tools/gemv_probe.hip, profiles/r01_gemv_probe.log): 2 on short rows, else 1; LN
  // variants 2-4 on wide N to amortise the per-block LayerNorm prologue
  // LN-fused: >= 2 rows per wave halves the blocks that each redo the row's LayerNorm
  // (profiles/r01_ln_rows_sweep.txt: 560m 1566 -> 1621 tok/s, 1b1 1229 -> 1242)
  const int R0 = !LN ? (K <= 2048 ? 2 : 1) : (N >= 12288 ? 4 : (N >= 2048 ? 2 : 1));
  rows_geometry(N, K, M, R0, R, waves);
  // U = 512-element chunks of a row in flight per iteration: an exact divisor of the row's chunk
  // count, so every row streams in whole rounds with no re-loaded tail (K = 1536 -> 3, 6144 -> 12,
  // 4096 -> 8, 16384 -> 8, 2560 -> 5, 1024 -> 2); fallback 4.
  const int cpr = K / 512;
  int u = (K % 512) ? 4 : (cpr <= 3 || cpr == 5 || cpr == 8 || cpr == 12) ? cpr
        : (cpr % 12 == 0 ? 12 : (cpr % 8 == 0 ? 8 : (cpr % 5 == 0 ? 5 : 4)));
  // wide blocks are bounded for 1024 threads (<= 128 VGPRs): keep the weight registers (R x U x 4 VGPRs)
  // small enough that nothing spills (LayerNorm / merge prologues hold ~32 more); 8 KB
  // per wave x up to 16 waves per CU is plenty in flight
  if (*waves > 4) {
    const int cap = (XM == X_PLAIN ? 12 : 8) / (M == 1 ? 1 : 2);  // measured spill-free (ISA metadata)
    while (*R * u > cap) u = (u % 2 == 0) ? u / 2 : (u > 4 ? 4 : u - 1);
  }
  *U = u;
}

template <int XM>
static bool gemv_rows_dispatch(const bf16* x, const LnArgs& ln, const AttnParts& pa, const bf16* w, int M, int N,
                               int K, const Epi& ep, hipStream_t s) {
  if (M > 4 || (K % 8) != 0 || K < 8 || (XM != X_PLAIN && K > 4096)) return false;
  // the tile GEMV takes the plain / LayerNorm-fused GEMVs of its token counts (tiles_take) when K has a tile path
  if ((XM == X_PLAIN || XM == X_LN) && ep.kind != EPI_ARGMAX && tiles_take(M, K) && (K % 64) == 0) return false;
  // M = 3..4: rows loses to the MFMA GEMV on LN-fused and large shapes
  // (tools/gemv_bench.hip, profiles/r01_gemv_bench_m4.log); keep it for small plain GEMVs and the head
  // (and for PARTS, which only this kernel implements).
  if (XM == X_PLAIN && M > 2 && ep.kind != EPI_ARGMAX && (size_t)N * K > (size_t)16 << 20) return false;
  if ((XM == X_LN || XM == X_EMB) && M > 2 && ep.kind != EPI_ARGMAX) return false;
  if (XM == X_EMB && (ep.kind == EPI_ARGMAX || (K % 4) != 0)) return false;
  // Tile choice from tools/gemv_bench.hip (profiles/r01_gemv_bench_m1_ur.log): U = 4 chunks of
  // every row in flight; the LN variants take 2-4 rows per wave on wide N to amortise the
  // per-block LayerNorm prologue; the head (argmax, 16 rows per block) keeps U = 2 on long K.
  if (ep.kind == EPI_ARGMAX) {  // a block = one 16-column tile
    if constexpr (XM == X_EMB) return false;
    else if (K <= 2048) {
      if (M == 1) gemv_rows_launch<4, 1, XM, 4>(x, ln, pa, w, M, N, K, ep, s);
      else if (M == 2) gemv_rows_launch<4, 2, XM, 4>(x, ln, pa, w, M, N, K, ep, s);
      else gemv_rows_launch<4, 4, XM, 4>(x, ln, pa, w, M, N, K, ep, s);
    } else {
      if (M == 1) gemv_rows_launch<4, 1, XM, 2>(x, ln, pa, w, M, N, K, ep, s);
      else if (M == 2) gemv_rows_launch<4, 2, XM, 2>(x, ln, pa, w, M, N, K, ep, s);
      else gemv_rows_launch<4, 4, XM, 2>(x, ln, pa, w, M, N, K, ep, s);
    }
    return true;
  }
  int R, waves, U;
  rows_plan(XM, M, N, K, &R, &waves, &U);
  auto go = [&](auto rc, auto uc) {
    constexpr int RR = decltype(rc)::value, UU = decltype(uc)::value;
    if (M == 1) gemv_rows_launch<RR, 1, XM, UU>(x, ln, pa, w, M, N, K, ep, s, waves);
    else if (M == 2) gemv_rows_launch<RR, 2, XM, UU>(x, ln, pa, w, M, N, K, ep, s, waves);
    else if constexpr (XM != X_EMB) gemv_rows_launch<RR, 4, XM, UU>(x, ln, pa, w, M, N, K, ep, s, waves);
  };
  auto gu = [&](auto rc) {
    switch (U) {
      case 1: go(rc, EpiKindC<1>{}); break;
      case 2: go(rc, EpiKindC<2>{}); break;
      case 3: go(rc, EpiKindC<3>{}); break;
      case 5: go(rc, EpiKindC<5>{}); break;
      case 8: go(rc, EpiKindC<8>{}); break;
      case 12: go(rc, EpiKindC<12>{}); break;
      default: go(rc, EpiKindC<4>{}); break;
    }
  };
  if (R == 1) gu(EpiKindC<1>{});
  else if (R == 2) gu(EpiKindC<2>{});
  else gu(EpiKindC<4>{});
  return true;
}

template <bool LN>
static void gemv_dispatch(const bf16* x, const LnArgs& ln, const bf16* w, int M, int N, int K, const Epi& ep,
                          hipStream_t s) {
  if (gemv_rows_dispatch<LN ? X_LN : X_PLAIN>(x, ln, AttnParts{}, w, M, N, K, ep, s)) return;
  if (!LN && gemv_tiles_dispatch(x, w, M, N, K, ep, s)) return;
  const int waves = gemv_waves(N, K);
  const bool two = M > 16;
  if (waves == 4) { if (two) gemv_launch<4, 2, LN>(x, ln, w, M, N, K, ep, s); else gemv_launch<4, 1, LN>(x, ln, w, M, N, K, ep, s); }
  else if (waves == 8) { if (two) gemv_launch<8, 2, LN>(x, ln, w, M, N, K, ep, s); else gemv_launch<8, 1, LN>(x, ln, w, M, N, K, ep, s); }
  else { if (two) gemv_launch<16, 2, LN>(x, ln, w, M, N, K, ep, s); else gemv_launch<16, 1, LN>(x, ln, w, M, N, K, ep, s); }
}

// LN(x) -> weight GEMM.  bf16 with M <= 8: LayerNorm fused into the GEMV prologue.  Otherwise a
// LayerNorm kernel writes the normalised activations to `xn_scratch` first.
void launch_linear_ln(int is_bf16, const float* x, int row_stride, int row_offset, const void* gamma,
                      const void* beta, float eps, void* xn_scratch, const void* W, int M, int N, int K,
                      const Epi& ep, hipStream_t s) {
  if (M <= 0) return;
  // the tile GEMV's token counts (tiles_take, up to 32): its LN-fused prologue where the shape allows it, else a
  // LayerNorm kernel + the tile GEMV (tools/gemv_probe.hip batched section)
  // the head (argmax) at M <= 2 keeps the rows GEMV's LayerNorm-fused argmax (profiles/r06_head_path_ab.txt: 3b / 7b1
  // B = 2 +0.4-0.6 % over the tile path; at M = 3..4 the tile path wins 1-3 %)
  const bool tiles = is_bf16 && tiles_take(M, K) && M <= 32 && (K % 64) == 0 && !(ep.kind == EPI_ARGMAX && M <= 2);
  if (is_bf16 && M <= 8 && (K % 8) == 0 && !tiles) {
    LnArgs ln{x, row_stride, row_offset, (const bf16*)gamma, (const bf16*)beta, eps};
    gemv_dispatch<true>(nullptr, ln, (const bf16*)W, M, N, K, ep, s);
    return;
  }
  if (tiles) {  // LN in the batched GEMV's prologue (gemv_ldsw4 LNS) where the shape allows it
    const LnArgs ln{x, row_stride, row_offset, (const bf16*)gamma, (const bf16*)beta, eps};
    if (gemv_tiles_dispatch<bf16>(nullptr, (const bf16*)W, M, N, K, ep, s, &ln)) return;
  }
  if (is_bf16 && K <= 4096 && (K % 4) == 0) {
    LnArgs ln{x, row_stride, row_offset, (const bf16*)gamma, (const bf16*)beta, eps};
    launch_ln_rows_wave(ln, M, K, (bf16*)xn_scratch, s);
  } else {
    launch_layernorm(is_bf16, x, nullptr, row_stride, row_offset, gamma, beta, xn_scratch, 0, M, K, eps, s);
  }
  launch_linear(is_bf16, xn_scratch, W, M, N, K, ep, s);
}

bool linear_parts_supported(int M, int K, int head_dim, int nsplit) {
  // M <= 2 defers the merge to the rows GEMV's prologue; at M = 3..4 the attention's last split merges by ticket
  // and the dense GEMV runs on the tile GEMV (round 6, profiles/r06_parts_max_m_ab.txt: 1024-token prompt, B = 4:
  // bloom-1b1 +2 %, 3b +8 %, 7b1 +16 %; B = 2 keeps the deferral, 3b -3 % without it).  BS_PARTS_MAX_M: A/B knob.
  static const int max_m = [] {
    const char* e = getenv("BS_PARTS_MAX_M");
    const int m = e ? atoi(e) : 0;
    return m >= 1 && m <= 4 ? m : 2;
  }();
  return M >= 1 && M <= max_m && K % 8 == 0 && K >= 8 && K <= 4096 && head_dim % 4 == 0 && nsplit >= 2 &&
         nsplit <= kPartsMaxSplit;
}

bool launch_linear_emb(const int* ids, const void* wemb, const void* emb_g, const void* emb_b, float* x_out,
                       const void* gamma, const void* beta, float eps, const void* W, int M, int N, int K,
                       const Epi& ep, hipStream_t s) {
  if (M < 1 || M > 2) return false;
  LnArgs ln{nullptr, 1, 0, (const bf16*)gamma, (const bf16*)beta, eps,
            ids, (const bf16*)wemb, (const bf16*)emb_g, (const bf16*)emb_b, x_out};
  return gemv_rows_dispatch<X_EMB>(nullptr, ln, AttnParts{}, (const bf16*)W, M, N, K, ep, s);
}

void launch_linear_parts(const AttnParts& p, const void* W, int M, int N, int K, const Epi& ep, hipStream_t s) {
  if (M <= 0) return;
  gemv_rows_dispatch<X_PARTS>(nullptr, LnArgs{}, p, (const bf16*)W, M, N, K, ep, s);
}

// Split-K factor of a 64x64-tile prefill GEMM: only the long-K shapes (fc2: K = 4h) gain from it -- KS
// about 768 / tiles (2..4 work items per CU), K / KS >= 1024 columns per split, the partials fitting the
// workspace; every other shape runs whole-K tiles (tools/gemm_splitk_bench.hip, profiles/r03_gemm_splitk.txt:
// bloom-1b1 fc2 at 512 tokens 31.8 -> 28.6 us with KS = 4, bloom-7b1 fc2 126.3 -> 122.8 with KS = 2; QKV,
// dense and fc1 only lose).
static int gemm_split_k(int M, int N, int K, const Epi& ep) {
  if (!ep.sk_ws || !ep.sk_tickets || K < 4096) return 1;
  const long tiles = (long)((M + 63) / 64) * ((N + 63) / 64);
  if (tiles > ep.sk_ntickets) return 1;
  for (int ks = 4; ks >= 2; ks--) {
    if (K % (ks * 64) || K / ks < 1024 || tiles * ks > 1024) continue;
    if ((size_t)tiles * ks * 64 * 64 > ep.sk_cap) continue;
    return ks;
  }
  return 1;
}

void launch_linear(int is_bf16, const void* X, const void* W, int M, int N, int K, const Epi& ep, hipStream_t s) {
  if (M <= 0) return;
  if (!is_bf16) {
    dim3 grid((N + 15) / 16, (M + 15) / 16);
    gemm_f32_kernel<<<grid, 256, 0, s>>>((const float*)X, (const float*)W, M, N, K, ep);
    return;
  }
  const bf16* x = (const bf16*)X;
  const bf16* w = (const bf16*)W;
  if (M <= 32) {
    gemv_dispatch<false>(x, LnArgs{}, w, M, N, K, ep, s);
    return;
  }
  if (M <= 64 && gemv_tiles_dispatch(x, w, M, N, K, ep, s)) return;
  if ((K % 64) == 0) {
    // 128x128 when it still gives every CU a block (>= 240 blocks), else 64x64, else 64x32
    auto blocks = [&](int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
    if (const int gb = gemm3_big_grid(M, N, K, ep)) {
      gemm3_launch<2, true, 256, 256>(x, w, M, N, K, ep, s, gb);
    } else if (const int gw = gemm3_wide_grid(M, N, K, ep)) {
      gemm3_launch<3, true, 256>(x, w, M, N, K, ep, s, gw);
    } else if (const int gp = gemm3_pair_grid(M, N, K, ep)) {
      gemm3_launch<2>(x, w, M, N, K, ep, s, gp);
    } else if (const int gn = gemm3_n96_grid(M, N, K, ep)) {
      gemm3_launch<3, true, 96>(x, w, M, N, K, ep, s, gn);
    } else if (const int g3 = gemm3_grid(M, N, K, ep)) {
      gemm3_launch(x, w, M, N, K, ep, s, g3);
    } else if (blocks(128, 128) >= 240) {
      gemm2_launch<128, 128, 1>(x, w, M, N, K, ep, s);
    } else if (blocks(64, 64) >= 128) {
      // below 240 128x128 tiles the K loop is latency-bound: 64x64 tiles with a 4-deep ring (beat 128x64,
      // profiles/r01_gemm_tile_sweep.txt, and 64x32 even at 192 tiles: bloom-1b1 dense 13.0 -> 12.4 us,
      // profiles/r03_gemm_splitk.txt), split-K for the long-K fc2 shapes
      gemm2_launch<64, 64, 4>(x, w, M, N, K, ep, s, gemm_split_k(M, N, K, ep));
    } else {
      // fewer than 128 64x64 tiles (a few hundred tokens of a narrow GEMM): 64x32 tiles for more blocks
      gemm2_launch<64, 32, 4>(x, w, M, N, K, ep, s);
    }
    return;
  }
  const long big = (long)((M + 127) / 128) * ((N + 127) / 128);
  if (big >= 256) {
    dim3 grid((N + 127) / 128, (M + 127) / 128);
    gemm_mfma_kernel<128, 128><<<grid, 256, 0, s>>>(x, w, M, N, K, ep);
  } else {
    dim3 grid((N + 63) / 64, (M + 63) / 64);
    gemm_mfma_kernel<64, 64><<<grid, 256, 0, s>>>(x, w, M, N, K, ep);
  }
}

// ------------------------------------------------------------------------------------
// Attention.  Scores = slope_h * key_pos + inv_norm * q.k (alibi.baddbmm, modeling_bloom.py
// :270-275), causal, fp32 softmax (:283), context = P.V (:292).
// ------------------------------------------------------------------------------------
// Decode (S == 1).  Block (head, row b, split) of WV waves; wave w of split sp takes the 64-position
// chunks c = w + WV*(sp + nsplit*j).  16 lanes cover one 8-dim slice each of a key/value row, so
// every load instruction reads 4 whole rows (coalesced); a chunk's K and V rows are requested
// before q is staged (they do not depend on it), so the first chunk's HBM round trip overlaps the
// q load.  Scores = ALiBi + q.k/sqrt(hd); online softmax across the wave's chunks; the wave
// partials merge through LDS.  nsplit == 1: the block writes ctx.  Otherwise it publishes a
// (max, sum, context) partial write-through (sc1) and takes a ticket; the block drawing the last
// ticket of its (row, head) merges all partials (sc1 loads, issued together) and writes ctx —
// MI355X_MICROARCH.md "Valid forms" row 1 (counter form, the last adder reads).

// The block body, also used by tools/attn_dense_fused.hip (the library passes done = nullptr): block (head, b, sp)
// of nsplit.  `done` (that experiment): the
// partials go out write-through (sc1) and, after every wave's stores drained, one lane adds 1 to *done (agent
// scope) -- MI355X_MICROARCH.md "Valid forms" row 1 (ONE lane of each storing workgroup, sc1 payload both sides).
template <typename T, int WV, int CH, bool SYNC = false>  // SYNC: the tool's `done` counter (compiled out otherwise)
__device__ __forceinline__ void attn_decode_block(const AttnArgs& a, int head, int b, int sp, int nsplit,
                                                  unsigned* done) {
  if constexpr (!SYNC) done = nullptr;
  constexpr int NI = CH / 4;  // load instructions per chunk (4 rows each)
  __shared__ __attribute__((aligned(16))) float qs[128];
  __shared__ float es[WV][64];
  __shared__ float pm[WV], pl[WV];
  __shared__ float pacc[WV][128];
  __shared__ int last;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hd = a.head_dim;
  const size_t rowbase = ((size_t)(a.slot + b) * a.n_head + head) * a.max_ctx;
  const T* kb = (const T*)a.k_cache + rowbase * hd;
  const T* vb = (const T*)a.v_cache + rowbase * hd;
  const int grp = lane >> 4, dl = lane & 15;
  const bool dval = dl * 8 < hd;
  const int doff = dval ? dl * 8 : 0;  // masked lanes re-read dims 0..7 (harmless)
  typedef typename Raw8<T>::type R8;
  R8 kr[NI], vr[NI];
  auto load_chunk = [&](int c, int lim) {
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int pr = min(c * CH + it * 4 + grp, lim);
      raw_load(kb + (size_t)pr * hd + doff, kr[it]);
    }
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int pr = min(c * CH + it * 4 + grp, lim);
      raw_load(vb + (size_t)pr * hd + doff, vr[it]);
    }
  };
  // The first chunk is requested before past_len is known (clamped to the cache, not the context:
  // positions past the context are masked to p = 0 below; the cache is zero-initialised and only
  // ever holds finite values, so their V rows contribute 0 * finite) and before q is staged.
  int c = w + WV * sp;
  if (c * CH < a.max_ctx) load_chunk(c, a.max_ctx - 1);
  // q, the slope and past_len are independent of each other: all in flight with the first chunk
  const float slope = a.slopes[head];
  const float qreg = threadIdx.x < hd ? to_f32(((const T*)a.q)[(size_t)b * a.hidden + head * hd + threadIdx.x]) : 0.f;
  const int past = a.past_dev ? a.past_dev[b] : a.past;
  const int nk = past + 1, nlast = nk - 1;
  const int nch = (nk + CH - 1) / CH;
  if (threadIdx.x < hd) qs[threadIdx.x] = qreg;  // hd <= 128 <= WV * 64
  __syncthreads();
  float qv[8];
  {
    const float4 q0 = *reinterpret_cast<const float4*>(&qs[doff]);
    const float4 q1 = *reinterpret_cast<const float4*>(&qs[doff + 4]);
    qv[0] = q0.x; qv[1] = q0.y; qv[2] = q0.z; qv[3] = q0.w; qv[4] = q1.x; qv[5] = q1.y; qv[6] = q1.z; qv[7] = q1.w;
  }
  float m_run = -INFINITY, l_run = 0.f;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (; c < nch; c += WV * nsplit) {
    if (c != w + WV * sp) load_chunk(c, nlast);
    float sc[NI];
#pragma unroll
    for (int it = 0; it < NI; it++) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < 8; j++) d += qv[j] * raw_get(kr[it], j);
      d = dval ? d : 0.f;
      d += dpp_f<0xB1>(d);   // sum over the row's 16 lanes (one DPP row): xor 1, xor 2,
      d += dpp_f<0x4E>(d);
      d += dpp_f<0x124>(d);  // rotate 4, rotate 8
      d += dpp_f<0x128>(d);
      sc[it] = d;
    }
    if (dl == 0) {
#pragma unroll
      for (int it = 0; it < NI; it++) es[w][it * 4 + grp] = sc[it];
    }
    __builtin_amdgcn_wave_barrier();
    const int p = c * CH + lane;
    const bool live = lane < CH && p < nk;
    const float s_me = live ? slope * (float)p + a.inv_norm * es[w][lane] : -INFINITY;
    const float m_new = fmaxf(m_run, wave_max(s_me));
    const float e = live ? __expf(s_me - m_new) : 0.f;
    const float scale = __expf(m_run - m_new);  // 0 on the first chunk (m_run = -inf)
    l_run = l_run * scale + wave_sum(e);
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] *= scale;
    m_run = m_new;
    __builtin_amdgcn_wave_barrier();
    es[w][lane] = e;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const float ep = es[w][it * 4 + grp];
#pragma unroll
      for (int j = 0; j < 8; j++) acc[j] += ep * raw_get(vr[it], j);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    acc[j] += __shfl_xor(acc[j], 16, 64);
    acc[j] += __shfl_xor(acc[j], 32, 64);
  }
  if (grp == 0 && dval) {
#pragma unroll
    for (int j = 0; j < 8; j++) pacc[w][dl * 8 + j] = acc[j];
  }
  if (lane == 0) { pm[w] = m_run; pl[w] = l_run; }
  __syncthreads();
  float M = -INFINITY, L = 0.f, o = 0.f;
  if (threadIdx.x < hd) {
    M = pm[0];
#pragma unroll
    for (int ww = 1; ww < WV; ww++) M = fmaxf(M, pm[ww]);
    if (M != -INFINITY) {  // a split past the context end holds no chunk
#pragma unroll
      for (int ww = 0; ww < WV; ww++) {
        const float wgt = __expf(pm[ww] - M);  // idle waves: exp(-inf) = 0
        L += wgt * pl[ww];
        o += wgt * pacc[ww][threadIdx.x];
      }
    }
  }
  T* ctx = (T*)a.ctx_out + (size_t)b * a.hidden + head * hd;
  if (nsplit == 1) {
    if (threadIdx.x < hd) ctx[threadIdx.x] = from_f32<T>(o / L);
    return;
  }
  const size_t pair = (size_t)(a.slot + b) * a.n_head + head;
  float* pacc_g = a.part_acc + pair * a.max_chunks * hd;  // [nsplit][hd]
  float* pml_g = a.part_ml + pair * a.max_chunks * 2;     // [nsplit][2]
  if (done) {  // tools/attn_dense_fused.hip: the same launch's dense blocks merge (attn_merge.h), sc1 both sides
    if (threadIdx.x < hd)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), attn_rsrc(pacc_g), (uint32_t)(sp * hd + threadIdx.x) * 4, 0, 16);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), attn_rsrc(pml_g), (uint32_t)sp * 8, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), attn_rsrc(pml_g), (uint32_t)sp * 8 + 4, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      typedef __attribute__((address_space(1))) unsigned gu32;
      __hip_atomic_fetch_add((gu32*)done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (a.defer_merge) {  // the consumer merges (attn_merge.h): plain stores, the kernel boundary publishes
    if (threadIdx.x < hd) pacc_g[sp * hd + threadIdx.x] = o;
    if (threadIdx.x == 0) { pml_g[sp * 2] = M; pml_g[sp * 2 + 1] = L; }
    return;
  }
  // ---- split partial (sc1 write-through), ticket, last arriver merges
  if (threadIdx.x < hd)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), attn_rsrc(pacc_g), (uint32_t)(sp * hd + threadIdx.x) * 4, 0, 16);
  if (threadIdx.x == 0) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), attn_rsrc(pml_g), (uint32_t)sp * 8, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), attn_rsrc(pml_g), (uint32_t)sp * 8 + 4, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    typedef __attribute__((address_space(1))) unsigned gu32;
    const unsigned old = __hip_atomic_fetch_add((gu32*)(a.tickets + pair), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (unsigned)(nsplit - 1);
    if (last) __hip_atomic_store((gu32*)(a.tickets + pair), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // one round trip: every thread takes all nsplit (m, l) pairs (same words in every lane) and its
  // context column of every split, all loads in flight together
  if (threadIdx.x < hd) {
    float mx = -INFINITY;
    float acc2 = 0.f, lsum = 0.f;
    for (int t0 = 0; t0 < nsplit; t0 += 16) {
      float m8[16], l8[16], o8[16];  // all of a group's loads in flight together
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int t = min(t0 + u, nsplit - 1);
        m8[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(pml_g), (uint32_t)t * 8, 0, 16));
        l8[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(pml_g), (uint32_t)t * 8 + 4, 0, 16));
        o8[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(attn_rsrc(pacc_g), (uint32_t)(t * hd + threadIdx.x) * 4, 0, 16));
      }
      // online merge of this group of 8 (duplicates past nsplit masked out)
      float gm = -INFINITY;
#pragma unroll
      for (int u = 0; u < 16; u++) gm = t0 + u < nsplit ? fmaxf(gm, m8[u]) : gm;
      const float nm = fmaxf(mx, gm);
      if (nm != -INFINITY) {
        const float sc = __expf(mx - nm);  // mx = -inf on the first group: 0
        acc2 *= sc;
        lsum *= sc;
#pragma unroll
        for (int u = 0; u < 16; u++) {
          if (t0 + u < nsplit && m8[u] != -INFINITY) {
            const float wgt = __expf(m8[u] - nm);
            acc2 += wgt * o8[u];
            lsum += wgt * l8[u];
          }
        }
        mx = nm;
      }
    }
    ctx[threadIdx.x] = from_f32<T>(acc2 / lsum);
  }
}

template <typename T, int WV, int CH = 64>  // CH: positions per wave chunk (64 or 32)
__global__ __launch_bounds__(WV * 64) void attn_decode_kernel(AttnArgs a) {
  attn_decode_block<T, WV, CH>(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.z, nullptr);
}

// S > 1: one wave per (query, head, row), online softmax over 64-key blocks.
template <typename T>
__global__ __launch_bounds__(64) void attn_prefill_kernel(AttnArgs a) {
  __shared__ float qs[128];
  const int t = blockIdx.x, head = blockIdx.y, b = blockIdx.z, lane = threadIdx.x;
  const int hd = a.head_dim;
  const int past = a.past_dev ? a.past_dev[b] : a.past;
  const int nk = past + t + 1;
  const int m = b * a.S + t;
  for (int d = lane; d < hd; d += 64) qs[d] = to_f32(((const T*)a.q)[(size_t)m * a.hidden + head * hd + d]);
  __syncthreads();
  const size_t rowbase = ((size_t)(a.slot + b) * a.n_head + head) * a.max_ctx;
  const T* kb = (const T*)a.k_cache + rowbase * hd;
  const T* vb = (const T*)a.v_cache + rowbase * hd;
  const float slope = a.slopes[head];
  float mrun = -INFINITY, l = 0.f, acc0 = 0.f, acc1 = 0.f;
  for (int c0 = 0; c0 < nk; c0 += 64) {
    const int j = c0 + lane;
    float s = -INFINITY;
    if (j < nk) {
      float dot = 0.f;
      for (int d = 0; d < hd; d += 8) {
        float kf[8];
        load8(kb + (size_t)j * hd + d, kf);
#pragma unroll
        for (int e = 0; e < 8; e++) dot += qs[d + e] * kf[e];
      }
      s = slope * (float)j + a.inv_norm * dot;
    }
    const float mn = fmaxf(mrun, wave_max(s));
    const float scale = __expf(mrun - mn);
    const float p = j < nk ? __expf(s - mn) : 0.f;
    l = l * scale + wave_sum(p);
    acc0 *= scale; acc1 *= scale;
    const int cnt = min(64, nk - c0);
    for (int jj = 0; jj < cnt; jj++) {
      const float pj = __shfl(p, jj, 64);
      const T* vr = vb + (size_t)(c0 + jj) * hd;
      if (lane < hd) acc0 += pj * to_f32(vr[lane]);
      if (lane + 64 < hd) acc1 += pj * to_f32(vr[lane + 64]);
    }
    mrun = mn;
  }
  T* o = (T*)a.ctx_out + (size_t)m * a.hidden + head * hd;
  const float inv = 1.0f / l;
  if (lane < hd) o[lane] = from_f32<T>(acc0 * inv);
  if (lane + 64 < hd) o[lane + 64] = from_f32<T>(acc1 * inv);
}

size_t attention_workspace_floats(int B, int n_head, int head_dim, int max_ctx, int* max_chunks, int* chunk) {
  const int ch = 64;  // == the wave width of attn_decode_kernel
  const int mc = (max_ctx + ch - 1) / ch;
  *max_chunks = mc;
  *chunk = ch;
  return (size_t)B * n_head * mc * (head_dim + 2);
}

// One 8-wave block per (row, head) when that already fills the chip or the cache is short;
// otherwise 4-wave blocks split the context so ~512 blocks stream the KV cache (>= one 64-position
// chunk per wave at full cache).  Static per (B, n_head, cache size), so the consumer of a deferred
// merge knows it without a device round trip.
// A wide variant (2-wave blocks of 32 positions, one block per 64 cached positions, ticket merge in the
// launch) measured bloom-7b1 B = 1 +1.7 %, bloom-1b1 B = 1 -4 % (profiles/r02_attn_wide_ab.txt): removed.
// Round 4 A/B (profiles/r04_attn_decode_splits_ab.txt): 2 or 1 chunks per split instead of 4 -- more blocks
// streaming the cache, more partials for the dense prologue to merge -- cost bloom-1b1 B = 1 3 %.
// Round 6 (profiles/r06_attn_splits_ab.txt, 1024-token prompt): ~512 blocks instead of ~256 when the pairs are few
// (bloom-1b1 B = 4 / 8 +1.6 / +3.8 %, 7b1 B = 4 +1.6 %); batch 1 stays bounded by the 4-chunk split length.
int attention_decode_splits(int B, int n_head, int max_chunks) {
  const int pairs = B * n_head;
  if (pairs >= 192 || max_chunks <= 4) return 1;
  const int nsplit = min((512 + pairs - 1) / pairs, (max_chunks + 3) / 4);
  return max(1, min(nsplit, 64));
}

void launch_attention(int is_bf16, const AttnArgs& a, hipStream_t s) {
  if (a.S == 1) {
    // Split partials merge either in the consumer (defer_merge, attn_merge.h) or, by ticket, in
    // the last split block of each (row, head) in this launch (no merge kernel either way).
    const int nsplit = attention_decode_splits(a.B, a.n_head, a.max_chunks);
    if (nsplit == 1) {
      dim3 g(a.n_head, a.B, 1);
      // the 8-wave block holds a CU (228 VGPRs: 2 waves per SIMD); above 256 (row, head) pairs, 4-wave
      // blocks run two per CU, so the grid takes half the rounds (bloom-1b1 B = 32: 512 pairs)
      if (is_bf16 && a.B * a.n_head > 256) attn_decode_kernel<bf16, 4><<<g, 256, 0, s>>>(a);
      else if (is_bf16) attn_decode_kernel<bf16, 8><<<g, 512, 0, s>>>(a);
      else attn_decode_kernel<float, 8><<<g, 512, 0, s>>>(a);
    } else if (is_bf16 && a.defer_merge) {
      // few (row, head) pairs: 8 waves x 32 positions per block, half the serial work per wave
      dim3 g(a.n_head, a.B, nsplit);
      attn_decode_kernel<bf16, 8, 32><<<g, 512, 0, s>>>(a);
    } else {
      dim3 g(a.n_head, a.B, nsplit);
      if (is_bf16) attn_decode_kernel<bf16, 4><<<g, 256, 0, s>>>(a);
      else attn_decode_kernel<float, 4><<<g, 256, 0, s>>>(a);
    }
  } else {
    if (is_bf16 && a.head_dim <= 128) {
      // split-KV: a query tile's keys over ceil(tiles / pf_tiles) blocks when the grid would leave CUs idle
      // and the partials fit (the longest query tile otherwise walks every key tile alone)
      attn_prefill_tr_launch(a, s);
    } else {
      dim3 g(a.S, a.n_head, a.B);
      if (is_bf16) attn_prefill_kernel<bf16><<<g, 64, 0, s>>>(a);
      else attn_prefill_kernel<float><<<g, 64, 0, s>>>(a);
    }
  }
}

// ------------------------------------------------------------------------------------
// past_adv (optional): row m's cached length advances by `seq` here, the step's last kernel (every
// reader of past_dev ran before it in stream order), so back-to-back decode steps need no set_past launch.
__global__ __launch_bounds__(1024) void argmax_finalize_kernel(const unsigned long long* keys, int ntiles,
                                                                const unsigned long long* keys_in,
                                                                unsigned long long* keys_out, int* tokens,
                                                                int* past_adv, int seq) {
  __shared__ unsigned long long sh[16];
  const int m = blockIdx.x;
  const unsigned long long* kr = keys + (size_t)m * ntiles;
  unsigned long long best = 0;
#pragma unroll 4
  for (int i = threadIdx.x; i < ntiles; i += 1024) {
    const unsigned long long k = kr[i];
    best = k > best ? k : best;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o, 64);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x < 64) {
    best = threadIdx.x < 16 ? sh[threadIdx.x] : 0ull;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      const unsigned long long other = __shfl_xor(best, o, 64);
      best = other > best ? other : best;
    }
    if (threadIdx.x == 0) {
      if (keys_in) best = keys_in[m] > best ? keys_in[m] : best;
      if (keys_out) keys_out[m] = best;
      if (tokens) tokens[m] = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
      if (past_adv) past_adv[m] += seq;
    }
  }
}

void launch_argmax_finalize(const unsigned long long* keys, int M, int ntiles, const unsigned long long* keys_in,
                            unsigned long long* keys_out, int* tokens, hipStream_t s, int* past_adv, int seq) {
  argmax_finalize_kernel<<<M, 1024, 0, s>>>(keys, ntiles, keys_in, keys_out, tokens, past_adv, seq);
}

// ------------------------------------------------------------------------------------
// Sequence-classification head (BS_FLAG_CLASSIFIER): logits[m][c] = xn[m] . score[c] (fp32 accumulation; no bias,
// BloomForSequenceClassification.score), class[m] = the first c of the largest logit (binary_classify,
// inference.cpp:57-69: a strict > scan).  n_labels <= 64 rows of K weights are a few KB: one 256-thread block per
// row, wave w takes labels w, w + 4, ...; each lane streams 16-B vectors of the row and the label.  The step's last
// kernel: advances past_adv[m] by seq like argmax_finalize.
template <typename T>
__global__ __launch_bounds__(256) void classify_kernel(const T* __restrict__ xn, const T* __restrict__ w, int n_labels,
                                                       int K, float* __restrict__ logits, int* __restrict__ cls,
                                                       int* past_adv, int seq) {
  __shared__ float lg[64];
  const int m = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const T* x = xn + (size_t)m * K;
  for (int c = wave; c < n_labels; c += 4) {
    const T* wr = w + (size_t)c * K;
    float acc = 0.f;
    for (int k = lane * 8; k < K; k += 64 * 8) {
      float xv[8], wv[8];
      load8(x + k, xv);
      load8(wr + k, wv);
#pragma unroll
      for (int j = 0; j < 8; j++) acc = fmaf(xv[j], wv[j], acc);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) lg[c] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    for (int c = 1; c < n_labels; c++)
      if (lg[c] > lg[best]) best = c;
    cls[m] = best;
    if (past_adv) past_adv[m] += seq;
  }
  if (logits)
    for (int c = threadIdx.x; c < n_labels; c += 256) logits[(size_t)m * n_labels + c] = lg[c];
}

void launch_classify(int is_bf16, const void* xn, const void* score, int M, int n_labels, int K, float* logits,
                     int* cls, int* past_adv, int seq, hipStream_t s) {
  if (is_bf16)
    classify_kernel<bf16><<<M, 256, 0, s>>>((const bf16*)xn, (const bf16*)score, n_labels, K, logits, cls, past_adv, seq);
  else
    classify_kernel<float><<<M, 256, 0, s>>>((const float*)xn, (const float*)score, n_labels, K, logits, cls, past_adv,
                                             seq);
}

// ------------------------------------------------------------------------------------
// Seeded top-k sampling, restating decoding::StaticDecoding (decoding.cpp:24-66) on the tile keys of
// the lm_head epilogue (key = order(logit) << 32 | vocab index: std::greater on (value, index)).
// One 1024-thread block per row.  (1) The top-k TILES by their max key: every element of the row's
// top-k lies in one of them (a tile outside holds an element below k tile maxima, i.e. below k
// elements).  (2) The top-k elements among those k x 16 logits.  (3) w_i = exp((l_i - l_0) / T),
// running sums in rank order, pick the first i with sum_{j<=i} w_j > u * sum(w) (u from the counter
// generator), else the last.  k rounds of a block-wide max, each removing the winner, do the
// selections; keys are unique (the index is in the key).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = __shfl_xor(v, o, 64);
    v = other > v ? other : v;
  }
  return v;
}

// Block-wide max over 1024 threads (sh: >= 17 words); every thread returns the max.
__device__ __forceinline__ unsigned long long block_max_u64(unsigned long long v, unsigned long long* sh) {
  v = wave_max_u64(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    unsigned long long t = threadIdx.x < (blockDim.x >> 6) ? sh[threadIdx.x] : 0ull;
    t = wave_max_u64(t);
    if (threadIdx.x == 0) sh[16] = t;
  }
  __syncthreads();
  const unsigned long long r = sh[16];
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint32_t sample_bits(uint64_t seed, uint32_t row, uint32_t pos) {
  const uint64_t key = d_sm64(seed ^ d_sm64(0x5A4D504C00000000ull | (uint64_t)row));
  return d_bits(key, pos);
}

__global__ __launch_bounds__(1024) void topk_sample_kernel(const unsigned long long* __restrict__ keys, int ntiles,
                                                           const float* __restrict__ logits, int ldl, int k,
                                                           float inv_temp, uint64_t seed, int slot,
                                                           const int* past_dev, int seq,
                                                           int* __restrict__ tokens, int* past_adv) {
  __shared__ unsigned long long sh[17];
  __shared__ unsigned long long pick[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  // (1) per-thread sorted top-16 of its tile keys, then k rounds of the block max
  unsigned long long loc[16];
#pragma unroll
  for (int j = 0; j < 16; j++) loc[j] = 0ull;
  const unsigned long long* kr = keys + (size_t)b * ntiles;
  for (int i = tid; i < ntiles; i += 1024) {
    unsigned long long key = kr[i];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const unsigned long long hi = key > loc[j] ? key : loc[j], lo = key > loc[j] ? loc[j] : key;
      loc[j] = hi;
      key = lo;
    }
  }
  for (int r = 0; r < k; r++) {
    const unsigned long long m = block_max_u64(loc[0], sh);
    if (tid == 0) pick[r] = m;
    if (loc[0] == m) {  // the unique owner drops its head
#pragma unroll
      for (int j = 0; j < 15; j++) loc[j] = loc[j + 1];
      loc[15] = 0ull;
    }
  }
  __syncthreads();
  // (2) the k x 16 candidate logits of those tiles, ranked by (value, index)
  unsigned long long cand = 0ull;
  if (tid < k * 16 && pick[tid >> 4] != 0ull) {
    const uint32_t col = ((uint32_t)(pick[tid >> 4] & 0xFFFFFFFFull) & ~15u) + (tid & 15);
    if ((int)col < ldl) cand = ((unsigned long long)f32_order_key(logits[(size_t)b * ldl + col]) << 32) | col;
  }
  __shared__ float pv[16];
  __shared__ int pi[16];
  for (int r = 0; r < k; r++) {
    const unsigned long long m = block_max_u64(cand, sh);
    if (cand == m && m != 0ull) {
      pv[r] = logits[(size_t)b * ldl + (uint32_t)(m & 0xFFFFFFFFull)];
      pi[r] = (int)(uint32_t)(m & 0xFFFFFFFFull);
      cand = 0ull;
    }
  }
  __syncthreads();
  // (3) weights, running sum, the draw
  if (tid == 0) {
    float w[16], sum = 0.f;
    for (int r = 0; r < k; r++) {
      w[r] = expf((pv[r] - pv[0]) * inv_temp);
      sum += w[r];
    }
    const int pos = past_dev[b] + seq;
    const float u = (float)(sample_bits(seed, (uint32_t)(slot + b), (uint32_t)pos) >> 8) * 0x1p-24f;
    const float target = u * sum;
    float run = 0.f;
    int sel = k - 1;
    for (int r = 0; r < k; r++) {
      run += w[r];
      if (run > target) { sel = r; break; }
    }
    tokens[b] = pi[sel];
    if (past_adv) past_adv[b] = pos;  // the only reader of past_dev[b] in this kernel is this thread
  }
}

void launch_topk_sample(const unsigned long long* keys, int ntiles, const float* logits, int ldl, int M, int k,
                        float inv_temp, uint64_t seed, int slot, const int* past_dev, int seq, int* tokens,
                        hipStream_t s, int* past_adv) {
  if (M > 0)
    topk_sample_kernel<<<M, 1024, 0, s>>>(keys, ntiles, logits, ldl, k, inv_temp, seed, slot, past_dev, seq, tokens,
                                          past_adv);
}

// Per-row cached positions, passed by value (graph-replayable: the kernels read the device copy).
struct PastRows { int v[64]; };
__global__ void set_past_kernel(int* p, PastRows r, int n) {
  if ((int)threadIdx.x < n) p[threadIdx.x] = r.v[threadIdx.x];
}
void launch_set_past(int* past_dev, const int* values, int n, hipStream_t s) {
  for (int i = 0; i < n; i += 64) {
    PastRows r;
    const int c = std::min(64, n - i);
    for (int j = 0; j < c; j++) r.v[j] = values[i + j];
    set_past_kernel<<<1, 64, 0, s>>>(past_dev + i, r, c);
  }
}

// ------------------------------------------------------------------------------------
// Weight-only int8 (BS_FLAG_INT8_WEIGHTS): the four block matrices of a bf16 stage held as int8
// [N][K] + one fp32 scale per output row -- the MI355X counterpart of the reference's bloom*-int8
// modules (server.py:796-799, data/Data.kt:19-30).  Rule (oracle/bloom_oracle.c or_quantize_int8
// restates it): scale[n] = max_k |W[n][k]| / 127 (1 for an all-zero row), Q[n][k] = rne(W[n][k] /
// scale[n]) clamped to [-127, 127], W = the bf16 weight the stage would otherwise hold.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quantize_rows_kernel(const bf16* __restrict__ W, int8_t* __restrict__ Q,
                                                            float* __restrict__ scale, int K) {
  const size_t row = blockIdx.x;
  const bf16* w = W + row * K;
  float amax = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) amax = fmaxf(amax, fabsf((float)w[k]));
  amax = wave_max(amax);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = amax > 0.f ? amax / 127.f : 1.f;  // IEEE division (no fast-math in this build)
  for (int k = threadIdx.x; k < K; k += 256) {
    const float v = fminf(fmaxf(rintf((float)w[k] / sc), -127.f), 127.f);
    Q[row * K + k] = (int8_t)(int)v;
  }
  if (threadIdx.x == 0) scale[row] = sc;
}

// out[n][k] = bf16(Q[n][k] * scale[n]) (scale null: Q itself, exact in bf16): operand of the bf16
// GEMM for prefill / wide batches, whose epilogue then applies the row scale (Epi::col_scale).
__global__ __launch_bounds__(256) void dequant_rows_kernel(const int8_t* __restrict__ Q, const float* __restrict__ scale,
                                                           bf16* __restrict__ out, size_t n8, int K) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    const size_t e = i * 8;
    const float sc = scale ? scale[e / K] : 1.f;
    const int2 q = *reinterpret_cast<const int2*>(Q + e);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int w = j < 4 ? q.x : q.y;
      const float v = (float)((w << (24 - 8 * (j & 3))) >> 24) * sc;  // sc = 1: exact Q
      o[j] = __builtin_bit_cast(unsigned short, (bf16)v);
    }
    *reinterpret_cast<u16x8*>(out + e) = o;
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Decode GEMV on int8 weights, M <= MM <= 8 rows.  A wave owns R weight rows; per step a lane
// streams 16 int8 weights (16 B, non-temporal) of each of its rows -- half the bytes of the bf16
// rows GEMV -- and reads the 16 matching bf16 activations of every row m (L2-resident).  fp32
// FMAs, DPP wave reduction, the row scale applied once to the reduced sum, then the usual epilogue.
template <int R, int MM, bool LN, int KIND, int CW, bool XL, int UQ, bool PARTS>
__device__ __forceinline__ void gemv_q8_body(const int8_t* __restrict__ Q, const float* __restrict__ scale,
                                             const bf16* __restrict__ Xg, const LnArgs& ln, const AttnParts& pa,
                                             int M, int N, int K, const Epi& ep) {
  // Offset form: u = q + 128 (one XOR per 4 weights) converts with v_cvt_f32_ubyte{0..3}, one op per
  // weight; sum_k x*q = sum_k x*u - 128 * sum_k x, the activation sum shared by the R rows.  The
  // FMAs run on float pairs (v_pk_fma_f32).
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * R;  // waves past N: row N-1, no store
  f2 acc[R][MM];
  f2 xs[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) {
    xs[m] = f2{0.f, 0.f};
#pragma unroll
    for (int r = 0; r < R; r++) acc[r][m] = f2{0.f, 0.f};
  }
  const int8_t* wr[R];
#pragma unroll
  for (int r = 0; r < R; r++) wr[r] = Q + (size_t)min(n0 + r, N - 1) * K;
  // CW bytes of each row per lane per step (16 or 32); UQ steps of every row in flight (the whole row up
  // to UQ * 64 * CW bytes: one round trip for a 1536- or 6144-column row, as the bf16 rows GEMV); the
  // loads are unconditional (clamped to the row; a step past the end is not computed)
  constexpr int W = CW / 16, STEP = 64 * CW;
  const int c0 = lane * CW;
  i32x4 wv[UQ][R][W];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < UQ; u++) {
      const int c = min(base + u * STEP, K - CW);
#pragma unroll
      for (int r = 0; r < R; r++)
#pragma unroll
        for (int w = 0; w < W; w++) wv[u][r][w] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wr[r] + c + 16 * w));
    }
  };
  // PARTS: the split-attention partials (attn_merge.h) go out before the weights
  const int kq = K >> 2, ngroups = M * kq;
  PartsRegs pr[PARTS ? 1 : 1];
  auto pld1 = [](const float* p, size_t i) { return p[i]; };
  auto pld4 = [](const float* p, size_t i) { return *reinterpret_cast<const float4*>(p + i); };
  if constexpr (PARTS) {
    const int g = min((int)threadIdx.x, ngroups - 1);
    attn_parts_load(pa, g / kq, (g % kq) * 4, pld1, pld4, pr[0]);
  }
  // LN: the rows (and gamma/beta) go out before the weights -- loads return in order, so rows issued
  // behind the weight stream would wait for all of it -- and the block normalises them into LDS while
  // the weight loads fly
  float4 xv[LN ? MM : 1][4];
  float cc[LN ? MM : 1];
  uint2 gb[4][2];
  if constexpr (LN) {
    if (threadIdx.x < 256) ln_rows_load<MM>(ln, M, K, xv, cc, gb);
  }
  // XL: the plain X rows likewise go out ahead of the weights (up to 4 16-B pieces per thread)
  constexpr int XP = XL ? 4 : 1;
  u16x8 xpre[XP];
  if constexpr (XL) {
#pragma unroll
    for (int j = 0; j < XP; j++) {
      const int i = min((int)threadIdx.x + j * (int)blockDim.x, M * K / 8 - 1);
      xpre[j] = reinterpret_cast<const u16x8*>(Xg)[i];
    }
  }
  issue(c0);
  extern __shared__ __align__(16) unsigned char q8_lds[];
  const bf16* X = Xg;
  if constexpr (LN) {
    __shared__ float scratch[64];
    ln_rows_finish<MM>(ln, M, K, xv, cc, gb, reinterpret_cast<bf16*>(q8_lds), scratch);
    X = reinterpret_cast<const bf16*>(q8_lds);
  } else if constexpr (PARTS) {  // merged context rows (bf16, the attn_decode_kernel rounding) to LDS
    bf16* xl = reinterpret_cast<bf16*>(q8_lds);
    auto put = [&](int g, const PartsRegs& rr) {
      float o[4];
      attn_parts_combine(pa.nsplit, rr, o);
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = (bf16)o[j];
      *reinterpret_cast<bf16x4*>(xl + (size_t)(g / kq) * K + (g % kq) * 4) = v;
    };
    if ((int)threadIdx.x < ngroups) put(threadIdx.x, pr[0]);
    for (int g = threadIdx.x + blockDim.x; g < ngroups; g += blockDim.x) {
      PartsRegs rr;
      attn_parts_load(pa, g / kq, (g % kq) * 4, pld1, pld4, rr);
      put(g, rr);
    }
    __syncthreads();
    X = xl;
  } else if (XL) {  // plain X staged once per block in LDS (the block's waves share it; one L2 pass)
    const int n16 = M * K / 8;
#pragma unroll
    for (int j = 0; j < XP; j++) {
      const int i = threadIdx.x + j * blockDim.x;
      if (i < n16) reinterpret_cast<u16x8*>(q8_lds)[i] = xpre[j];
    }
    for (int i = threadIdx.x + XP * blockDim.x; i < n16; i += blockDim.x)
      reinterpret_cast<u16x8*>(q8_lds)[i] = reinterpret_cast<const u16x8*>(Xg)[i];
    __syncthreads();
    X = reinterpret_cast<const bf16*>(q8_lds);
  }
  for (int base = c0; base < K; base += UQ * STEP) {
    const bool more = base + UQ * STEP < K;
#pragma unroll
    for (int u = 0; u < UQ; u++) {
      if (base + u * STEP >= K) continue;
#pragma unroll
      for (int w = 0; w < W; w++) {
        const int cw = base + u * STEP + 16 * w;
        i32x4 cur[R];
#pragma unroll
        for (int r = 0; r < R; r++) cur[r] = wv[u][r][w];
        if (more) {  // step u of the next round replaces it in flight
          const int c = min(base + (UQ + u) * STEP, K - CW);
#pragma unroll
          for (int r = 0; r < R; r++)
            wv[u][r][w] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wr[r] + c + 16 * w));
        }
        f2 wf[R][8];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint32_t uq = (uint32_t)cur[r][i] ^ 0x80808080u;
            wf[r][2 * i] = f2{(float)(uq & 0xFF), (float)((uq >> 8) & 0xFF)};
            wf[r][2 * i + 1] = f2{(float)((uq >> 16) & 0xFF), (float)(uq >> 24)};
          }
#pragma unroll
        for (int m = 0; m < MM; m++) {
          if (m < M) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 a0 = *reinterpret_cast<const u32x4*>(X + (size_t)m * K + cw);
            const u32x4 a1 = *reinterpret_cast<const u32x4*>(X + (size_t)m * K + cw + 8);
            f2 xf[8];
#pragma unroll
            for (int i = 0; i < 4; i++) {
              xf[i] = f2{__uint_as_float(a0[i] << 16), __uint_as_float(a0[i] & 0xFFFF0000u)};
              xf[4 + i] = f2{__uint_as_float(a1[i] << 16), __uint_as_float(a1[i] & 0xFFFF0000u)};
            }
#pragma unroll
            for (int i = 0; i < 8; i++) xs[m] += xf[i];
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
              for (int i = 0; i < 8; i++) acc[r][m] = __builtin_elementwise_fma(xf[i], wf[r][i], acc[r][m]);
          }
        }
      }
    }
  }
  float mine = 0.f;
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int m = 0; m < MM; m++) {
      if (m < M) {
        const float t = wave_sum((acc[r][m].x + acc[r][m].y) - 128.f * (xs[m].x + xs[m].y));
        if (lane == r * MM + m) mine = t;
      }
    }
  const int r = lane / MM, m = lane - r * MM;
  if (lane < R * MM && m < M && n0 + r < N) epi_store<bf16, KIND>(ep, m, n0 + r, mine);  // ep.col_scale = scale
}

// WIDE: one block of up to 16 waves per CU (the rows GEMV's per-CU geometry, rows_geometry): the
// LayerNorm / merge prologue runs once per CU instead of once per 4 waves, and narrow N still spreads
// over every CU.
template <int R, int MM, bool LN, int CW, bool XL = false, int UQ = 2, bool PARTS = false, bool WIDE = false>
__global__ __launch_bounds__(WIDE ? 1024 : 256) void gemv_q8_kernel(const int8_t* __restrict__ Q, const float* __restrict__ scale,
                                                      const bf16* __restrict__ X, LnArgs ln, AttnParts pa, int M,
                                                      int N, int K, Epi ep) {
  epi_dispatch(ep.kind, [&](auto kc) {
    if constexpr (decltype(kc)::value != EPI_ARGMAX)
      gemv_q8_body<R, MM, LN, decltype(kc)::value, CW, XL, UQ, PARTS>(Q, scale, X, ln, pa, M, N, K, ep);
  });
}

template <int R, int MM, bool LN = false, bool PARTS = false>
static void gemv_q8_launch(const int8_t* Q, const float* scale, const bf16* X, const LnArgs& ln, int M, int N, int K,
                           const Epi& ep, hipStream_t s, const AttnParts& pa = AttnParts{}) {
  const size_t shm = (LN || PARTS) ? (size_t)M * K * sizeof(bf16) : 0;
  const int blocks = (N + 4 * R - 1) / (4 * R);
  // steps of every row in flight: the whole row (<= 8 steps of 64 x 16 B) for matrices up to 12 M weights,
  // where the grid is a few waves per SIMD and latency decides (bloom-1b1 int8 B=1: 1207 -> 1221 tok/s);
  // one step beyond, where the stream is bandwidth-bound and deeper queues only cost occupancy
  // (bloom-7b1 int8: UQ=1 486.6, UQ=2 471.7, the whole row 454 tok/s; profiles/r02_q8_uq_ab.txt)
  const int steps = (K + 1023) / 1024;
  const int uq = (size_t)N * K > (12u << 20) ? 1 : min(steps <= 2 ? 2 : steps <= 4 ? 4 : steps <= 6 ? 6 : 8, R >= 4 ? 4 : 8);
  // plain X staged in LDS (loaded ahead of the weights) by the wide blocks when it fits 64 KB
  const bool wide_xl = (size_t)M * K * sizeof(bf16) <= 65536;
  if constexpr (MM == 1 && R <= 2) {
    int rr = 0, waves = 0;
    rows_geometry(N, K, M, R, &rr, &waves);
    // matrices up to 32 M weights (bloom-1b1 int8 B=1 1206 -> 1281 tok/s, 560m 1685 -> 1768, 3b 735 -> 762;
    // bloom-7b1's 50-67 M-weight QKV / fc1 / fc2 keep 4-wave blocks; profiles/r02_q8_uq_ab.txt)
    if ((size_t)N * K <= (32u << 20) && rr <= 2 && waves >= 4 && uq <= 6) {
      auto go = [&](auto rc) {
        constexpr int RW = decltype(rc)::value;
        const int wb = (N + waves * RW - 1) / (waves * RW);
        const dim3 g(wb), t(waves * 64);
        if constexpr (!LN && !PARTS) {
          if (wide_xl) {  // plain X staged in LDS, loaded ahead of the weights
            const size_t shx = (size_t)M * K * sizeof(bf16);
            if (uq == 1) gemv_q8_kernel<RW, 1, false, 16, true, 1, false, true><<<g, t, shx, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
            else if (uq <= 2) gemv_q8_kernel<RW, 1, false, 16, true, 2, false, true><<<g, t, shx, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
            else if (uq <= 4) gemv_q8_kernel<RW, 1, false, 16, true, 4, false, true><<<g, t, shx, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
            else gemv_q8_kernel<RW, 1, false, 16, true, 6, false, true><<<g, t, shx, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
            return;
          }
        }
        if (uq == 1) gemv_q8_kernel<RW, 1, LN, 16, false, 1, PARTS, true><<<g, t, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
        else if (uq <= 2) gemv_q8_kernel<RW, 1, LN, 16, false, 2, PARTS, true><<<g, t, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
        else if (uq <= 4) gemv_q8_kernel<RW, 1, LN, 16, false, 4, PARTS, true><<<g, t, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
        else gemv_q8_kernel<RW, 1, LN, 16, false, 6, PARTS, true><<<g, t, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
      };
      if (rr == 2) go(EpiKindC<2>{});
      else go(EpiKindC<1>{});
      return;
    }
  }
  if (uq == 1) {  // one step in flight
    gemv_q8_kernel<R, MM, LN, 16, false, 1, PARTS><<<blocks, 256, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
  } else if (uq <= 2) {
    gemv_q8_kernel<R, MM, LN, 16, false, 2, PARTS><<<blocks, 256, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
  } else if (uq <= 4) {
    gemv_q8_kernel<R, MM, LN, 16, false, 4, PARTS><<<blocks, 256, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
  } else if (uq <= 6) {
    gemv_q8_kernel<R, MM, LN, 16, false, 6, PARTS><<<blocks, 256, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
  } else {
    gemv_q8_kernel<R, MM, LN, 16, false, 8, PARTS><<<blocks, 256, shm, s>>>(Q, scale, X, ln, pa, M, N, K, ep);
  }
}

bool linear_q8_gemv(int M, int K) { return M >= 1 && M <= 8 && K % 32 == 0; }

// Rows per wave of the int8 GEMV: 2 (profiles/r01_q8_rows_sweep.txt: 1b1 B=1 1128 -> 1177 tok/s against 1 row
// below N = 8192, 7b1 equal).
bool linear_q8_ln_fused(int M, int K) { return M >= 1 && M <= 4 && K % 32 == 0 && K <= 4096; }

void launch_linear_q8_ln(const float* x, int row_stride, int row_offset, const void* gamma, const void* beta,
                         float eps, const int8_t* Q, const float* scale, int M, int N, int K, const Epi& ep,
                         hipStream_t s) {
  Epi e = ep;
  e.col_scale = scale;
  const LnArgs ln{x, row_stride, row_offset, (const bf16*)gamma, (const bf16*)beta, eps};
  if (M <= 1) gemv_q8_launch<2, 1, true>(Q, scale, nullptr, ln, M, N, K, e, s);
  else if (M <= 2) gemv_q8_launch<2, 2, true>(Q, scale, nullptr, ln, M, N, K, e, s);
  else gemv_q8_launch<2, 4, true>(Q, scale, nullptr, ln, M, N, K, e, s);
}

bool linear_q8_parts_supported(int M, int K, int head_dim, int nsplit) {
  return M >= 1 && M <= 2 && K % 32 == 0 && K <= 4096 && head_dim % 4 == 0 && nsplit >= 2 && nsplit <= kPartsMaxSplit;
}

void launch_linear_q8_parts(const AttnParts& p, const int8_t* Q, const float* scale, int M, int N, int K,
                            const Epi& ep, hipStream_t s) {
  Epi e = ep;
  e.col_scale = scale;
  if (M <= 1) gemv_q8_launch<2, 1, false, true>(Q, scale, nullptr, LnArgs{}, M, N, K, e, s, p);
  else gemv_q8_launch<2, 2, false, true>(Q, scale, nullptr, LnArgs{}, M, N, K, e, s, p);
}

void launch_quantize_rows(const void* W_bf16, int8_t* Q, float* scale, int N, int K, hipStream_t s) {
  if (N > 0) quantize_rows_kernel<<<N, 256, 0, s>>>((const bf16*)W_bf16, Q, scale, K);
}

void launch_dequant_rows(const int8_t* Q, const float* scale, void* out_bf16, int N, int K, hipStream_t s) {
  const size_t n8 = (size_t)N * K / 8;
  const int blocks = (int)std::min<size_t>((n8 + 255) / 256, 8192);
  if (n8) dequant_rows_kernel<<<blocks, 256, 0, s>>>(Q, scale, (bf16*)out_bf16, n8, K);
}

void launch_ln_rows(const float* x, int row_stride, int row_offset, const void* gamma, const void* beta, float eps,
                    void* out_bf16, int M, int K, hipStream_t s) {
  if (K <= 4096 && (K % 4) == 0) {
    LnArgs ln{x, row_stride, row_offset, (const bf16*)gamma, (const bf16*)beta, eps};
    launch_ln_rows_wave(ln, M, K, (bf16*)out_bf16, s);
  } else {
    launch_layernorm(1, x, nullptr, row_stride, row_offset, gamma, beta, out_bf16, 0, M, K, eps, s);
  }
}

void launch_linear_q8(const void* X, const int8_t* Q, const float* scale, void* w_scratch, int M, int N, int K,
                      const Epi& ep, hipStream_t s) {
  if (M <= 0) return;
  if (ep.kind == EPI_ARGMAX) abort();  // the tied lm_head stays bf16
  const bf16* x = (const bf16*)X;
  Epi e = ep;
  e.col_scale = scale;
  // batched decode (4 < M <= 32): the int8 gemv_ldsw4 / tile GEMV converts in registers (no dequant pass);
  // at M = 8 it reads the weights once where gemv_q8 re-reads activations per row (bloom-7b1 int8 B=8)
  if (M > 4 && M <= 32 && gemv_tiles_dispatch<int8_t>(x, Q, M, N, K, e, s)) return;
  if (linear_q8_gemv(M, K)) {
    const LnArgs ln{};
    if (M <= 1) gemv_q8_launch<2, 1>(Q, scale, x, ln, M, N, K, e, s);
    else if (M <= 2) gemv_q8_launch<2, 2>(Q, scale, x, ln, M, N, K, e, s);
    else if (M <= 4) gemv_q8_launch<2, 4>(Q, scale, x, ln, M, N, K, e, s);
    else gemv_q8_launch<1, 8>(Q, scale, x, ln, M, N, K, e, s);
    return;
  }
  // prefill: dequantize to the bf16 scratch, then the bf16 GEMM
  launch_dequant_rows(Q, nullptr, w_scratch, N, K, s);
  launch_linear(1, X, w_scratch, M, N, K, e, s);
}
