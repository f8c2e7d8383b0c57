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
#include "common.h"
#include "kernels.h"

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
  return kind == 2 ? __fadd_rn(1.0f, t) : t;
}

template <typename T>
__global__ void gen_fill_kernel(T* dst, uint64_t n, uint64_t key, uint64_t key2, int kind) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = from_f32<T>(d_gen_value(kind, key, key2, (uint32_t)i));
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

void launch_gen_fill(void* dst, int is_bf16, uint64_t n, uint64_t key, int kind, hipStream_t s) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return;
  if (is_bf16)
    gen_fill_kernel<bf16><<<(unsigned)blocks, 256, 0, s>>>((bf16*)dst, n, key, h_sm64(key), kind);
  else
    gen_fill_kernel<float><<<(unsigned)blocks, 256, 0, s>>>((float*)dst, n, key, h_sm64(key), kind);
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
  unsigned long long key = valid ? (((unsigned long long)f32_order_key(v) << 32) | (0xFFFFFFFFu - (uint32_t)n)) : 0ull;
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) {
    unsigned long long other = __shfl_xor(key, o, 64);
    key = other > key ? other : key;
  }
  if (valid && (n & 15) == 0) e.keys[(size_t)m * ntiles + (n >> 4)] = key;
  if (valid && e.logits) e.logits[(size_t)m * e.ldo + n] = v;
}

template <typename T>
__device__ __forceinline__ void epi_store(const Epi& e, int m, int n, float v) {
  switch (e.kind) {
    case EPI_QKV: {
      v += to_f32(((const T*)e.bias)[n]);
      const int three = 3 * e.head_dim;
      const int head = n / three, r = n - head * three, which = r / e.head_dim, d = r - which * e.head_dim;
      if (which == 0) {
        e.q_out[(size_t)m * e.hidden + head * e.head_dim + d] = v;
      } else {
        const int b = m / e.seq, t = m - b * e.seq;
        const int past = e.past_dev ? *e.past_dev : e.past;
        const size_t idx = (((size_t)(e.slot + b) * e.n_head + head) * e.max_ctx + past + t) * e.head_dim + d;
        T* c = (T*)(which == 1 ? e.k_cache : e.v_cache);
        c[idx] = from_f32<T>(v);
      }
      break;
    }
    case EPI_RESID: {
      const size_t i = (size_t)m * e.ldo + n;
      e.out_f32[i] = (v + to_f32(((const T*)e.bias)[n])) + e.resid[i];
      break;
    }
    case EPI_GELU: {
      ((T*)e.out_act)[(size_t)m * e.ldo + n] = from_f32<T>(gelu_bloom(v + to_f32(((const T*)e.bias)[n])));
      break;
    }
    default: break;
  }
}

// ------------------------------------------------------------------------------------
// gemv_mfma: out[m][n] for M <= 16*MT rows.  Block = one 16-column tile of W, WAVES waves
// split K; each wave streams its K range of the 16 weight rows straight to VGPRs (16 B per
// lane, U k-steps in flight) and runs one v_mfma_f32_16x16x32_bf16 per k-step and m-tile
// with A = W tile (rows = n), B = X^T (cols = m).  Partial tiles meet in LDS.
// ------------------------------------------------------------------------------------
template <int WAVES, int MT, int U>
__global__ __launch_bounds__(WAVES * 64) void gemv_mfma_kernel(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                                               int M, int N, int K, Epi ep) {
  __shared__ float red[WAVES][MT * 16][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const bf16* wp = W + (size_t)min(n0 + r, N - 1) * K + g * 8;
  const bf16* xp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) xp[mt] = X + (size_t)min(mt * 16 + r, M - 1) * K + g * 8;
  const int ksteps = K >> 5;
  const int per = (ksteps + WAVES - 1) / WAVES;
  const int s0 = w * per, s1 = min(ksteps, s0 + per);
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + U <= s1; s += U) {
    bf16x8 a[U], b[MT][U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = *reinterpret_cast<const bf16x8*>(wp + (size_t)(s + u) * 32);
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
      for (int u = 0; u < U; u++) b[mt][u] = *reinterpret_cast<const bf16x8*>(xp[mt] + (size_t)(s + u) * 32);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int mt = 0; mt < MT; mt++) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[mt][u], acc[mt], 0, 0, 0);
  }
  for (; s < s1; ++s) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(wp + (size_t)s * 32);
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      bf16x8 b = *reinterpret_cast<const bf16x8*>(xp[mt] + (size_t)s * 32);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[mt], 0, 0, 0);
    }
  }
  // D[row = 4g+i (n)][col = r (m)]
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int i = 0; i < 4; i++) red[w][mt * 16 + r][4 * g + i] = acc[mt][i];
  __syncthreads();
  const int ntiles = (N + 15) >> 4;
  for (int t = threadIdx.x; t < MT * 256; t += WAVES * 64) {
    const int ml = t >> 4, nl = t & 15;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ww++) v += red[ww][ml][nl];
    const int m = ml, n = n0 + nl;
    const bool valid = m < M && n < N;
    if (ep.kind == EPI_ARGMAX) argmax_tile16(ep, m, n, v, valid, ntiles);
    else if (valid) epi_store<bf16>(ep, m, n, v);
  }
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
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int m = m0 + wm * (BM / 2) + i * 16 + 4 * g + e;
        const int n = n0 + wn * (BN / 2) + j * 16 + r;
        const bool valid = m < M && n < N;
        if (ep.kind == EPI_ARGMAX) argmax_tile16(ep, m, n, acc[i][j][e], valid, ntiles);
        else if (valid) epi_store<bf16>(ep, m, n, acc[i][j][e]);
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
  const bool valid = m < M && n < N;
  if (ep.kind == EPI_ARGMAX) argmax_tile16(ep, m, n, acc, valid, (N + 15) >> 4);
  else if (valid) epi_store<float>(ep, m, n, acc);
}

template <int WAVES, int MT>
static void gemv_launch(const bf16* X, const bf16* W, int M, int N, int K, const Epi& ep, hipStream_t s) {
  gemv_mfma_kernel<WAVES, MT, 8><<<(N + 15) / 16, WAVES * 64, 0, s>>>(W, X, M, N, K, ep);
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
    const int ntiles = (N + 15) / 16, ksteps = K / 32;
    int waves = 4;
    while (waves < 16 && ntiles * waves < 2048 && waves * 2 <= ksteps) waves *= 2;
    const bool two = M > 16;
    if (waves == 4) { if (two) gemv_launch<4, 2>(x, w, M, N, K, ep, s); else gemv_launch<4, 1>(x, w, M, N, K, ep, s); }
    else if (waves == 8) { if (two) gemv_launch<8, 2>(x, w, M, N, K, ep, s); else gemv_launch<8, 1>(x, w, M, N, K, ep, s); }
    else { if (two) gemv_launch<16, 2>(x, w, M, N, K, ep, s); else gemv_launch<16, 1>(x, w, M, N, K, ep, s); }
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
// Decode (S == 1): block = (chunk c, head, row b); 16 lanes per key row (8 dims each),
// 16 keys per pass; writes the chunk's (max, sum, unnormalised context).
template <typename T>
__global__ __launch_bounds__(256) void attn_decode_partial_kernel(AttnArgs a) {
  __shared__ float sc[256];
  __shared__ float red[16][129];
  __shared__ float sh[4];
  const int c = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int past = a.past_dev ? *a.past_dev : a.past;
  const int nk = past + 1;
  const int p0 = c * a.chunk;
  if (p0 >= nk) return;
  const int p1 = min(nk, p0 + a.chunk);
  const int tid = threadIdx.x, grp = tid >> 4, dl = tid & 15;
  const int hd = a.head_dim;
  const bool dval = dl * 8 < hd;
  float q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (dval) load8(a.q + (size_t)b * a.hidden + head * hd + dl * 8, q);
  const size_t rowbase = ((size_t)(a.slot + b) * a.n_head + head) * a.max_ctx;
  const T* kb = (const T*)a.k_cache + rowbase * hd;
  const T* vb = (const T*)a.v_cache + rowbase * hd;
  const float slope = a.slopes[head];
  for (int p = p0 + grp; p < p1; p += 16) {
    float kf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dval) load8(kb + (size_t)p * hd + dl * 8, kf);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) s += q[j] * kf[j];
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (dl == 0) sc[p - p0] = slope * (float)p + a.inv_norm * s;
  }
  __syncthreads();
  const int n = p1 - p0;
  float mx = -INFINITY;
  for (int j = tid; j < n; j += 256) mx = fmaxf(mx, sc[j]);
  mx = wave_max(mx);
  if ((tid & 63) == 0) sh[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  float l = 0.f;
  for (int j = tid; j < n; j += 256) { float e = __expf(sc[j] - mx); sc[j] = e; l += e; }
  l = block_sum_256(l, sh);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int p = p0 + grp; p < p1; p += 16) {
    if (dval) {
      float vf[8];
      load8(vb + (size_t)p * hd + dl * 8, vf);
      const float pv = sc[p - p0];
#pragma unroll
      for (int j = 0; j < 8; j++) acc[j] += pv * vf[j];
    }
  }
  if (dval) {
#pragma unroll
    for (int j = 0; j < 8; j++) red[grp][dl * 8 + j] = acc[j];
  }
  __syncthreads();
  const size_t pidx = ((size_t)b * a.n_head + head) * a.max_chunks + c;
  if (tid < hd) {
    float o = 0.f;
#pragma unroll
    for (int gg = 0; gg < 16; gg++) o += red[gg][tid];
    a.part_acc[pidx * hd + tid] = o;
  }
  if (tid == 0) { a.part_ml[pidx * 2] = mx; a.part_ml[pidx * 2 + 1] = l; }
}

template <typename T>
__global__ __launch_bounds__(128) void attn_decode_combine_kernel(AttnArgs a) {
  const int head = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int past = a.past_dev ? *a.past_dev : a.past;
  const int nch = (past + 1 + a.chunk - 1) / a.chunk;
  const size_t base = ((size_t)b * a.n_head + head) * a.max_chunks;
  float M = -INFINITY;
  for (int c = 0; c < nch; c++) M = fmaxf(M, a.part_ml[(base + c) * 2]);
  float L = 0.f, o = 0.f;
  for (int c = 0; c < nch; c++) {
    const float wgt = __expf(a.part_ml[(base + c) * 2] - M);
    L += wgt * a.part_ml[(base + c) * 2 + 1];
    if (d < a.head_dim) o += wgt * a.part_acc[(base + c) * a.head_dim + d];
  }
  if (d < a.head_dim) ((T*)a.ctx_out)[(size_t)b * a.hidden + head * a.head_dim + d] = from_f32<T>(o / L);
}

// S > 1: one wave per (query, head, row), online softmax over 64-key blocks.
template <typename T>
__global__ __launch_bounds__(64) void attn_prefill_kernel(AttnArgs a) {
  __shared__ float qs[128];
  const int t = blockIdx.x, head = blockIdx.y, b = blockIdx.z, lane = threadIdx.x;
  const int hd = a.head_dim;
  const int past = a.past_dev ? *a.past_dev : a.past;
  const int nk = past + t + 1;
  const int m = b * a.S + t;
  for (int d = lane; d < hd; d += 64) qs[d] = a.q[(size_t)m * a.hidden + head * hd + d];
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
  const int ch = 64;
  const int mc = (max_ctx + ch - 1) / ch;
  *max_chunks = mc;
  *chunk = ch;
  return (size_t)B * n_head * mc * (head_dim + 2);
}

void launch_attention(int is_bf16, const AttnArgs& a, hipStream_t s) {
  if (a.S == 1) {
    dim3 g1(a.max_chunks, a.n_head, a.B), g2(a.n_head, a.B);
    if (is_bf16) {
      attn_decode_partial_kernel<bf16><<<g1, 256, 0, s>>>(a);
      attn_decode_combine_kernel<bf16><<<g2, 128, 0, s>>>(a);
    } else {
      attn_decode_partial_kernel<float><<<g1, 256, 0, s>>>(a);
      attn_decode_combine_kernel<float><<<g2, 128, 0, s>>>(a);
    }
  } else {
    dim3 g(a.S, a.n_head, a.B);
    if (is_bf16) attn_prefill_kernel<bf16><<<g, 64, 0, s>>>(a);
    else attn_prefill_kernel<float><<<g, 64, 0, s>>>(a);
  }
}

// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void argmax_finalize_kernel(const unsigned long long* keys, int* tokens, int ntiles) {
  __shared__ unsigned long long sh[4];
  const int m = blockIdx.x;
  unsigned long long best = 0;
  for (int i = threadIdx.x; i < ntiles; i += 256) {
    unsigned long long k = keys[(size_t)m * ntiles + i];
    best = k > best ? k : best;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    unsigned long long other = __shfl_xor(best, o, 64);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; i++) best = sh[i] > best ? sh[i] : best;
    tokens[m] = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
  }
}

void launch_argmax_finalize(const unsigned long long* keys, int* tokens, int M, int ntiles, hipStream_t s) {
  argmax_finalize_kernel<<<M, 256, 0, s>>>(keys, tokens, ntiles);
}

__global__ void set_past_kernel(int* p, int v) { *p = v; }
void launch_set_past(int* past_dev, int value, hipStream_t s) { set_past_kernel<<<1, 1, 0, s>>>(past_dev, value); }
