// decode_engine.hip — persistent decode step of one BLOOM pipeline stage (see decode_engine.h).
//
// Math per layer restated from HF BLOOM (modeling_bloom.py; oracle/bloom_oracle.c header has the
// line map): LN_in (:359-403 block order), fused QKV with the per-head interleave [heads][3][hd]
// (:214-217), ALiBi + q.k/sqrt(hd), fp32 softmax, P.V (:245-310), dense + residual, LN_post,
// fc1 + tanh-GELU (:111-121), fc2 + residual (:313-340); last stage ln_f + tied lm_head (:536,
// :561-566) + greedy argmax.  This is what the reference's ONNX sub-model of one stage computes
// (inference::run_inference, inference.cpp:145-218).
//
// Hand-off protocol (MI355X_MICROARCH.md "Valid forms", row 1; cdna_hip_programming.md
// Guideline 16): every byte another workgroup reads in this launch is stored write-through
// (buffer store sc1) and loaded sc1 (L1 bypass); every storing wave drains vmcnt(0), the
// workgroup meets at a barrier, then one lane adds 1 to the edge counter (agent scope, sharded
// over 8 lines).  A consumer's wave 0 polls the 8 shards relaxed, with a 200 ms give-up that sets
// the error words so every waiting workgroup leaves; the last workgroup of the launch re-zeroes
// all counters, so a launch starts from zero without a memset node.
#include "common.h"
#include "decode_engine.h"

#include <cstdio>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

namespace {

// The per-layer pointer table is immutable during a launch: read it through the constant address
// space so it lands in SGPRs (a generic-pointer load is treated as divergent and turns every
// buffer descriptor built from it into a waterfall loop).
typedef __attribute__((address_space(4))) const uint64_t cu64;
__device__ __forceinline__ DeLayer layer_at(const DeArgs& a, int l) {
  constexpr int NW = sizeof(DeLayer) / 8;
  static_assert(sizeof(DeLayer) == NW * 8, "DeLayer is a table of pointers");
  const cu64* p = (const cu64*)a.layers + (size_t)l * NW;
  uint64_t w[NW];
#pragma unroll
  for (int i = 0; i < NW; i++) w[i] = p[i];
  return __builtin_bit_cast(DeLayer, w);
}

constexpr int NT = 512, NWV = 8;
constexpr int SHARDS = 8, SHARD_STRIDE = 16;          // counter shards, 64 B apart
constexpr uint64_t TIMEOUT_TICKS = 20000000ull;       // 200 ms of the 100 MHz s_memrealtime clock
enum { E_QKV = 0, E_ATT = 1, E_DENSE = 2, E_FC1 = 3, E_FC2 = 4, E_PER_LAYER = 5 };

// ---- sc1 (write-through / L1-bypass) accesses through buffer descriptors with a uniform base
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
__device__ __forceinline__ u32x4 ld16(const void* base, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off, 0, 16);
}
__device__ __forceinline__ uint32_t ld4(const void* base, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st4(void* base, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st2(void* base, uint32_t off, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st16(void* base, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), off, 0, 16);
}
__device__ __forceinline__ uint16_t bf_bits(float v) { return __builtin_bit_cast(uint16_t, (bf16)v); }
__device__ __forceinline__ float bf_f(const bf16* p, int i) { return (float)p[i]; }

__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[0], a[1]}, (bf16x2){b[0], b[1]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[2], a[3]}, (bf16x2){b[2], b[3]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[4], a[5]}, (bf16x2){b[4], b[5]}, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[6], a[7]}, (bf16x2){b[6], b[7]}, acc, false);
  return acc;
}

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ void split_rows(int N, int& r0, int& r1) {
  r0 = (int)(((long long)blockIdx.x * N) / gridDim.x);
  r1 = (int)(((long long)(blockIdx.x + 1) * N) / gridDim.x);
}
// Every workgroup publishes every GEMV edge (an empty row slice included), so a GEMV edge is
// complete when all gridDim.x workgroups have arrived.
__device__ __forceinline__ unsigned producers(int) { return gridDim.x; }

// ---- edge counters
// A give-up aborts the launch: err makes every other wait fail at once, every workgroup skips to
// the final ticket (so the last one still re-zeroes the state), err_log keeps the code for the host.
__device__ __forceinline__ void fail_launch(const DeArgs& a, unsigned code) {
  __hip_atomic_store((gu32*)a.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_or((gu32*)a.err_log, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 polls until the edge counter reaches `target`; all waves meet at a barrier after.
// Returns false (uniformly) when the launch failed or this wait timed out.
__device__ __forceinline__ bool wg_wait(const DeArgs& a, int edge, unsigned target, int* flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    const gu32* c = (const gu32*)(a.ctr + (size_t)edge * SHARDS * SHARD_STRIDE);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      unsigned v = lane < SHARDS ? __hip_atomic_load(c + lane * SHARD_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const unsigned e = lane == SHARDS ? __hip_atomic_load((const gu32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v = __shfl(v, 0, 64);
      if (__any(e != 0u)) { ok = false; break; }
      if (v >= target) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > TIMEOUT_TICKS) {
        if (lane == 0) fail_launch(a, 0x100u + (unsigned)edge);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) *flag = ok ? 1 : 0;
  }
  __syncthreads();
  // readfirstlane: the result is wave-uniform, so control flow and the loop-carried stream state
  // after a wait stay scalar (an LDS-loaded bool would make them divergent)
  return __builtin_amdgcn_readfirstlane(*(volatile int*)flag) != 0;
}

// Every storing wave drains its write-through stores; then one lane signals the edge.
__device__ __forceinline__ void wg_publish(const DeArgs& a, int edge) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add((gu32*)(a.ctr + ((size_t)edge * SHARDS + (blockIdx.x & (SHARDS - 1))) * SHARD_STRIDE), 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- weight stream of one GEMV phase: wave w owns rows r0 + w + 8i of the workgroup's slice and
// walks them in 512-element (1 KB per wave instruction) chunks; loads past the end re-read the
// last chunk so the refill loop issues a fixed count.
struct WS {
  const bf16* base;     // first row of the workgroup's slice (wave-uniform)
  uint32_t off;         // byte offset of the next chunk to load (wave-uniform)
  uint32_t row_off;     // byte offset of the row holding it
  uint32_t row_step;    // bytes between this wave's consecutive rows (8 rows)
  int cpr, n, nl, lkc;  // chunks per row, chunks of this wave, load cursor
  int K;
};

__device__ __forceinline__ void ws_init(WS& s, const bf16* W, int K, int r0, int r1) {
  const int wv = wave_id();
  s.K = K;
  s.cpr = K >> 9;
  const int nr = r1 - r0 - wv;
  s.n = nr > 0 ? ((nr + NWV - 1) / NWV) * s.cpr : 0;
  s.base = W + (size_t)r0 * K;
  s.row_off = (uint32_t)wv * K * 2;
  s.off = s.row_off;
  s.row_step = (uint32_t)NWV * K * 2;
  s.nl = 0; s.lkc = 0;
}

// buffer load: lane offset in a VGPR, chunk offset in an SGPR (all cursor math is scalar);
// aux 2 = nt (weights are read once per step)
template <bool NTW>
__device__ __forceinline__ bf16x8 ws_load(WS& s) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rsrc(s.base), (threadIdx.x & 63) * 16, s.off, NTW ? 2 : 0);
  if (s.nl + 1 < s.n) {
    s.nl++;
    if (++s.lkc == s.cpr) { s.lkc = 0; s.row_off += s.row_step; s.off = s.row_off; }
    else s.off += 1024;
  }
  return __builtin_bit_cast(bf16x8, u);
}

template <int P, bool NTW>
__device__ __forceinline__ void ws_prefetch(WS& s, bf16x8 (&ring)[P]) {
  // every slot is (re)defined here, so the ring is dead between a phase's last use and this call
#pragma unroll
  for (int u = 0; u < P; u++) {
    if (u < s.n) ring[u] = ws_load<NTW>(s);
    else ring[u] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// Consume the wave's chunks against the activations in LDS (xs [MM][K] bf16); row sums go to
// res[m][row_local].  Same accumulation order as gemv_rows_kernel (per lane over the chunks of a
// row, then a wave reduction).
template <int MM, int P, bool NTW>
__device__ __forceinline__ void ws_consume(WS& s, bf16x8 (&ring)[P], const bf16* xs, int M, float* res, int maxrows) {
  const int n = s.n;
  if (n == 0) return;
  const int lane = threadIdx.x & 63, wv = wave_id();
  const int K = s.K, cpr = s.cpr;
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) acc[m] = 0.f;
  int ci = 0, ckc = 0;
  auto use = [&](const bf16x8& wv8) {
    const int koff = ckc * 512 + lane * 8;
#pragma unroll
    for (int m = 0; m < MM; m++) {
      const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + m * K + koff);
      acc[m] = dot8(wv8, xv, acc[m]);
    }
    if (++ckc == cpr) {
      ckc = 0;
#pragma unroll
      for (int m = 0; m < MM; m++) {
        const float v = wave_sum(acc[m]);
        acc[m] = 0.f;
        if (lane == 0 && m < M) res[m * maxrows + wv + NWV * ci] = v;
      }
      ci++;
    }
  };
  int j = 0;
  for (; j + 2 * P <= n; j += P) {  // steady state: every refill valid, P loads in flight
#pragma unroll
    for (int u = 0; u < P; u++) {
      use(ring[u]);
      ring[u] = ws_load<NTW>(s);
    }
  }
#pragma unroll
  for (int u = 0; u < P; u++) {
    if (j + u < n) {
      use(ring[u]);
      if (j + u + P < n) ring[u] = ws_load<NTW>(s);
    }
  }
#pragma unroll
  for (int u = 0; u < P; u++)
    if (j + P + u < n) use(ring[u]);
}

// ---- activation rows in registers: thread t holds elements [4i, 4i+4) for i = t, t + 512
template <int MM>
struct Rows {
  float4 v[MM][2];
};

template <int MM>
__device__ __forceinline__ void rows_load_f32(Rows<MM>& r, const float* x, int M, int K) {
#pragma unroll
  for (int m = 0; m < MM; m++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int i = threadIdx.x + NT * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M && i * 4 < K) {
        const u32x4 u = ld16(x, (uint32_t)((m * K + i * 4) * 4));
        v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
      }
      r.v[m][j] = v;
    }
}

// word_embeddings rows ids[m] (bf16 table, never written in a launch: plain loads)
template <int MM>
__device__ __forceinline__ void rows_load_emb(Rows<MM>& r, const bf16* wemb, const int* ids, int M, int K) {
#pragma unroll
  for (int m = 0; m < MM; m++) {
    const bf16* row = wemb + (size_t)(m < M ? ids[m] : 0) * K;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int i = threadIdx.x + NT * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M && i * 4 < K) {
        const uint2 u = *reinterpret_cast<const uint2*>(row + i * 4);
        v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
                        __uint_as_float(u.y & 0xFFFF0000u));
      }
      r.v[m][j] = v;
    }
  }
}

template <int MM>
__device__ __forceinline__ void block_sum(float (&v)[MM], float* scr) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int m = 0; m < MM; m++) v[m] = wave_sum(v[m]);
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < MM; m++) scr[wv * MM + m] = v[m];
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MM; m++) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; w++) t += scr[w * MM + m];
    v[m] = t;
  }
  __syncthreads();
}

// nn.LayerNorm in place (biased variance, eps inside the sqrt), gamma/beta bf16
template <int MM>
__device__ __forceinline__ void rows_ln(Rows<MM>& r, int K, const bf16* g, const bf16* b, float eps, float* scr) {
  float s[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) {
    s[m] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; j++) s[m] += (r.v[m][j].x + r.v[m][j].y) + (r.v[m][j].z + r.v[m][j].w);
  }
  block_sum<MM>(s, scr);
  float mean[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) {
    mean[m] = s[m] / (float)K;
    s[m] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      if ((threadIdx.x + NT * j) * 4 < K) {
        const float d0 = r.v[m][j].x - mean[m], d1 = r.v[m][j].y - mean[m], d2 = r.v[m][j].z - mean[m],
                    d3 = r.v[m][j].w - mean[m];
        s[m] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
  }
  block_sum<MM>(s, scr);
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int i = threadIdx.x + NT * j;
    if (i * 4 < K) {
      const uint2 graw = *reinterpret_cast<const uint2*>(g + i * 4);
      const uint2 braw = *reinterpret_cast<const uint2*>(b + i * 4);
      const float gg[4] = {__uint_as_float(graw.x << 16), __uint_as_float(graw.x & 0xFFFF0000u),
                           __uint_as_float(graw.y << 16), __uint_as_float(graw.y & 0xFFFF0000u)};
      const float bb[4] = {__uint_as_float(braw.x << 16), __uint_as_float(braw.x & 0xFFFF0000u),
                           __uint_as_float(braw.y << 16), __uint_as_float(braw.y & 0xFFFF0000u)};
#pragma unroll
      for (int m = 0; m < MM; m++) {
        const float rstd = 1.0f / sqrtf(s[m] / (float)K + eps);
        float4& v = r.v[m][j];
        v.x = (v.x - mean[m]) * rstd * gg[0] + bb[0];
        v.y = (v.y - mean[m]) * rstd * gg[1] + bb[1];
        v.z = (v.z - mean[m]) * rstd * gg[2] + bb[2];
        v.w = (v.w - mean[m]) * rstd * gg[3] + bb[3];
      }
    }
  }
}

template <int MM>
__device__ __forceinline__ void rows_to_xs(const Rows<MM>& r, int K, bf16* xs) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int m = 0; m < MM; m++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int i = threadIdx.x + NT * j;
      if (i * 4 < K) {
        const float4 v = r.v[m][j];
        *reinterpret_cast<bf16x4*>(xs + m * K + i * 4) = (bf16x4){(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
      }
    }
}

// bf16 [M][K] handed-off activations -> LDS
__device__ __forceinline__ void stage_bf16(const bf16* src, int M, int K, bf16* xs) {
  const int nv = M * K / 8;
  for (int i = threadIdx.x; i < nv; i += NT) *reinterpret_cast<u32x4*>(xs + i * 8) = ld16(src, (uint32_t)i * 16);
}

// ---- attention unit (row b, head, split sp of nsplit over the 64-position chunks [c0, c1))
// 8 waves take the chunks round-robin; same per-chunk math as attn_decode_kernel.
__device__ __forceinline__ void attn_unit(const DeArgs& a, const DeLayer& W, int b, int head, int c0, int c1, float* scr, float* outm,
                          float* outl, float* outacc) {
  float* qs = scr;               // [128]
  float* es = scr + 128;         // [8][64]
  float* pm = scr + 640;         // [8]
  float* pl = scr + 648;         // [8]
  float* pacc = scr + 656;       // [8][128]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int hd = a.hd;
  const int nk = a.past + 1, nlast = nk - 1;
  if (threadIdx.x < hd / 2) {
    const uint32_t u = ld4(a.q, (uint32_t)((b * a.h + head * hd) * 2 + threadIdx.x * 4));
    qs[2 * threadIdx.x] = __uint_as_float(u << 16);
    qs[2 * threadIdx.x + 1] = __uint_as_float(u & 0xFFFF0000u);
  }
  __syncthreads();
  const size_t rowbase = ((size_t)(a.slot + b) * a.nh + head) * a.max_ctx * hd;
  const bf16* kb = W.kc + rowbase;
  const bf16* vb = W.vc + rowbase;
  const float slope = a.slopes[head];
  const int grp = lane >> 4, dl = lane & 15;
  const bool dval = dl * 8 < hd;
  const int doff = dval ? dl * 8 : 0;
  float qv[8];
#pragma unroll
  for (int j = 0; j < 8; j++) qv[j] = qs[doff + j];
  float m_run = -INFINITY, l_run = 0.f;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int c = c0 + wv; c < c1; c += NWV) {
    u32x4 kr[16], vr[16];
#pragma unroll
    for (int it = 0; it < 16; it++) {
      const int pr = min(c * 64 + it * 4 + grp, nlast);
      kr[it] = ld16(kb, (uint32_t)((pr * hd + doff) * 2));
    }
#pragma unroll
    for (int it = 0; it < 16; it++) {
      const int pr = min(c * 64 + it * 4 + grp, nlast);
      vr[it] = ld16(vb, (uint32_t)((pr * hd + doff) * 2));
    }
    float sc[16];
#pragma unroll
    for (int it = 0; it < 16; it++) {
      const uint32_t w4[4] = {kr[it].x, kr[it].y, kr[it].z, kr[it].w};
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        d += qv[2 * j] * __uint_as_float(w4[j] << 16);
        d += qv[2 * j + 1] * __uint_as_float(w4[j] & 0xFFFF0000u);
      }
      d = dval ? d : 0.f;
      d += __shfl_xor(d, 8, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      sc[it] = d;
    }
    if (dl == 0) {
#pragma unroll
      for (int it = 0; it < 16; it++) es[wv * 64 + it * 4 + grp] = sc[it];
    }
    __builtin_amdgcn_wave_barrier();
    const int p = c * 64 + lane;
    const bool live = p < nk;
    const float s_me = live ? slope * (float)p + a.inv_norm * es[wv * 64 + lane] : -INFINITY;
    const float m_new = fmaxf(m_run, wave_max(s_me));
    const float e = live ? __expf(s_me - m_new) : 0.f;
    const float scale = __expf(m_run - m_new);
    l_run = l_run * scale + wave_sum(e);
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] *= scale;
    m_run = m_new;
    __builtin_amdgcn_wave_barrier();
    es[wv * 64 + lane] = e;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 16; it++) {
      const float ep = es[wv * 64 + it * 4 + grp];
      const uint32_t w4[4] = {vr[it].x, vr[it].y, vr[it].z, vr[it].w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        acc[2 * j] += ep * __uint_as_float(w4[j] << 16);
        acc[2 * j + 1] += ep * __uint_as_float(w4[j] & 0xFFFF0000u);
      }
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
    for (int j = 0; j < 8; j++) pacc[wv * 128 + dl * 8 + j] = acc[j];
  }
  if (lane == 0) { pm[wv] = m_run; pl[wv] = l_run; }
  __syncthreads();
  if (threadIdx.x < hd) {
    float Mx = pm[0];
#pragma unroll
    for (int w = 1; w < NWV; w++) Mx = fmaxf(Mx, pm[w]);
    float L = 0.f, o = 0.f;
    if (Mx != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NWV; w++) {
        const float wgt = __expf(pm[w] - Mx);
        L += wgt * pl[w];
        o += wgt * pacc[w * 128 + threadIdx.x];
      }
    }
    outacc[threadIdx.x] = o;
    if (threadIdx.x == 0) { *outm = Mx; *outl = L; }
  }
  __syncthreads();
}

// ---- diagnostics: one s_memrealtime stamp per phase boundary per workgroup (trace == null: off)
#define STAMP(k)                                                                           \
  do {                                                                                     \
    if (a.trace && threadIdx.x == 0)                                                       \
      a.trace[(size_t)blockIdx.x * a.trace_stride + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// ---- the kernel
template <int MM, int P, bool NTW>
__global__ __launch_bounds__(512) void decode_engine_kernel(DeArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);
  float* res = reinterpret_cast<float*>(smem + a.lds_res);
  float* scr = reinterpret_cast<float*>(smem + a.lds_scr);  // 8 KB
  int* flag = reinterpret_cast<int*>(scr + 1900);
  const int tid = threadIdx.x;
  const int nwg = gridDim.x, wg = blockIdx.x;
  const int M = a.M, h = a.h, nh = a.nh, hd = a.hd, L = a.L, maxrows = a.maxrows;
  const int first = a.ids != nullptr;

  int q0, q1, d0, d1, f0, f1, hr0 = 0, hr1 = 0;
  split_rows(3 * h, q0, q1);
  split_rows(h, d0, d1);
  split_rows(4 * h, f0, f1);
  if (a.has_head) split_rows(a.head_rows, hr0, hr1);

  WS ws;
  bf16x8 ring[P];
  ws_init(ws, layer_at(a, 0).wqkv, h, q0, q1);
  ws_prefetch<P, NTW>(ws, ring);

  auto xout_of = [&](int l) -> float* {
    if (l == L - 1 && a.x_out) return a.x_out;
    return (l & 1) ? a.xb1 : a.xb0;
  };

  STAMP(0);
  for (int l = 0; l < L; l++) {
    const DeLayer W = layer_at(a, l);
    const float* xin = l == 0 ? (first ? a.x0 : a.x_in) : xout_of(l - 1);
    float* xo = xout_of(l);
    // ================= LN_in + QKV
    if (l > 0 && !wg_wait(a, (l - 1) * E_PER_LAYER + E_FC2, producers(h), flag)) goto done;
    STAMP(1 + l * 12 + 0);
    {
      Rows<MM> r;
      if (l == 0 && first) {
        rows_load_emb<MM>(r, a.wemb, a.ids, M, h);
        rows_ln<MM>(r, h, a.emb_g, a.emb_b, a.eps, scr);
        // this workgroup reads back x0 only for its own dense rows [d0, d1) (residual of layer 0)
#pragma unroll
        for (int m = 0; m < MM; m++)
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const int i = tid + NT * j;
            const float vv[4] = {r.v[m][j].x, r.v[m][j].y, r.v[m][j].z, r.v[m][j].w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const int k = i * 4 + e;
              if (m < M && k >= d0 && k < d1) st4(a.x0, (uint32_t)((m * h + k) * 4), __float_as_uint(vv[e]));
            }
          }
      } else {
        rows_load_f32<MM>(r, xin, M, h);
      }
      rows_ln<MM>(r, h, W.ln1_g, W.ln1_b, a.eps, scr);
      rows_to_xs<MM>(r, h, xs);
    }
    __syncthreads();
    ws_consume<MM, P, NTW>(ws, ring, xs, M, res, maxrows);
    STAMP(1 + l * 12 + 1);
    __syncthreads();
    {
      const int nr = q1 - q0;
      for (int t = tid; t < M * nr; t += NT) {
        const int m = t / nr, rl = t - m * nr, n = q0 + rl;
        const float v = res[m * maxrows + rl] + bf_f(W.bqkv, n);
        const int three = 3 * hd, head = n / three, rr = n - head * three, which = rr / hd, d = rr - which * hd;
        if (which == 0) {
          st2(a.q, (uint32_t)((m * h + head * hd + d) * 2), bf_bits(v));
        } else {
          const size_t idx = (((size_t)(a.slot + m) * nh + head) * a.max_ctx + a.past) * hd + d;
          // V = K + kv_half_bytes: one uniform descriptor base for both caches
          st2(W.kc, (uint32_t)(idx * 2) + (which == 2 ? a.kv_half_bytes : 0u), bf_bits(v));
        }
      }
    }
    wg_publish(a, l * E_PER_LAYER + E_QKV);
    STAMP(1 + l * 12 + 2);

    // ================= attention (units = rows x heads x context splits)
    if (!wg_wait(a, l * E_PER_LAYER + E_QKV, producers(3 * h), flag)) goto done;
    STAMP(1 + l * 12 + 3);
    {
      const int nk = a.past + 1, nch = (nk + 63) >> 6;
      int nsplit = nwg / (M * nh);
      nsplit = max(1, min(nsplit, nch));
      const int units = M * nh * nsplit;
      for (int u = wg; u < units; u += nwg) {
        const int bh = u / nsplit, sp = u - bh * nsplit, b = bh / nh, head = bh - b * nh;
        const int c0 = (int)(((long long)sp * nch) / nsplit), c1 = (int)(((long long)(sp + 1) * nch) / nsplit);
        float* oacc = scr + 1696;   // [128], after attn_unit's scratch (ends at 1680)
        float* stats = scr + 1840;  // m, l
        attn_unit(a, W, b, head, c0, c1, scr, stats, stats + 1, oacc);
        bool merger = nsplit == 1;
        if (!merger) {
          // publish this split's partial, take a ticket; the last split of (b, head) merges
          float* pp = a.part;
          const uint32_t base = (uint32_t)u * (hd + 2) * 4;
          if (tid < hd) st4(pp, base + (2 + tid) * 4, __float_as_uint(oacc[tid]));
          if (tid == 0) { st4(pp, base, __float_as_uint(stats[0])); st4(pp, base + 4, __float_as_uint(stats[1])); }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) {
            gu32* tk = (gu32*)(a.tick + ((size_t)l * 4 + b) * nh + head);
            const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = old == (unsigned)(nsplit - 1);
          }
          __syncthreads();
          merger = __builtin_amdgcn_readfirstlane(*(volatile int*)flag) != 0;
          if (merger && tid < hd) {
            const int u0 = bh * nsplit;
            float Mx = -INFINITY;
            for (int s2 = 0; s2 < nsplit; s2++)
              Mx = fmaxf(Mx, __uint_as_float(ld4(pp, (uint32_t)(u0 + s2) * (hd + 2) * 4)));
            float Ls = 0.f, o = 0.f;
            for (int s2 = 0; s2 < nsplit; s2++) {
              const uint32_t bs = (uint32_t)(u0 + s2) * (hd + 2) * 4;
              const float mm = __uint_as_float(ld4(pp, bs));
              if (mm == -INFINITY) continue;
              const float wgt = __expf(mm - Mx);
              Ls += wgt * __uint_as_float(ld4(pp, bs + 4));
              o += wgt * __uint_as_float(ld4(pp, bs + (2 + tid) * 4));
            }
            oacc[tid] = o;
            if (tid == 0) stats[1] = Ls;
          }
          __syncthreads();
        }
        if (merger) {
          if (tid < hd) st2(a.ctx, (uint32_t)((b * h + head * hd + tid) * 2), bf_bits(oacc[tid] / stats[1]));
          if (!(nsplit == 1) && tid == 0)  // ticket back to zero for the next launch
            __hip_atomic_store((gu32*)(a.tick + ((size_t)l * 4 + b) * nh + head), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          wg_publish(a, l * E_PER_LAYER + E_ATT);
        }
      }
    }

    STAMP(1 + l * 12 + 4);
    // ================= dense + residual
    ws_init(ws, W.wo, h, d0, d1);
    ws_prefetch<P, NTW>(ws, ring);
    if (!wg_wait(a, l * E_PER_LAYER + E_ATT, (unsigned)(M * nh), flag)) goto done;
    STAMP(1 + l * 12 + 5);
    stage_bf16(a.ctx, M, h, xs);
    __syncthreads();
    ws_consume<MM, P, NTW>(ws, ring, xs, M, res, maxrows);
    STAMP(1 + l * 12 + 6);
    __syncthreads();
    {
      const int nr = d1 - d0;
      for (int t = tid; t < M * nr; t += NT) {
        const int m = t / nr, rl = t - m * nr, n = d0 + rl;
        const float resid = __uint_as_float(ld4(xin, (uint32_t)((m * h + n) * 4)));
        const float v = (res[m * maxrows + rl] + bf_f(W.bo, n)) + resid;
        st4(a.attn, (uint32_t)((m * h + n) * 4), __float_as_uint(v));
      }
    }
    wg_publish(a, l * E_PER_LAYER + E_DENSE);
    STAMP(1 + l * 12 + 7);

    // ================= LN_post + fc1 + GELU
    ws_init(ws, W.w1, h, f0, f1);
    ws_prefetch<P, NTW>(ws, ring);
    if (!wg_wait(a, l * E_PER_LAYER + E_DENSE, producers(h), flag)) goto done;
    STAMP(1 + l * 12 + 8);
    {
      Rows<MM> r;
      rows_load_f32<MM>(r, a.attn, M, h);
      rows_ln<MM>(r, h, W.ln2_g, W.ln2_b, a.eps, scr);
      rows_to_xs<MM>(r, h, xs);
    }
    __syncthreads();
    ws_consume<MM, P, NTW>(ws, ring, xs, M, res, maxrows);
    __syncthreads();
    {
      const int nr = f1 - f0;
      for (int t = tid; t < M * nr; t += NT) {
        const int m = t / nr, rl = t - m * nr, n = f0 + rl;
        const float v = gelu_bloom(res[m * maxrows + rl] + bf_f(W.b1, n));
        st2(a.g, (uint32_t)((m * 4 * h + n) * 2), bf_bits(v));
      }
    }
    wg_publish(a, l * E_PER_LAYER + E_FC1);
    STAMP(1 + l * 12 + 9);

    // ================= fc2 + residual
    ws_init(ws, W.w2, 4 * h, d0, d1);
    ws_prefetch<P, NTW>(ws, ring);
    if (!wg_wait(a, l * E_PER_LAYER + E_FC1, producers(4 * h), flag)) goto done;
    STAMP(1 + l * 12 + 10);
    stage_bf16(a.g, M, 4 * h, xs);
    __syncthreads();
    ws_consume<MM, P, NTW>(ws, ring, xs, M, res, maxrows);
    __syncthreads();
    {
      const int nr = d1 - d0;
      for (int t = tid; t < M * nr; t += NT) {
        const int m = t / nr, rl = t - m * nr, n = d0 + rl;
        const float resid = __uint_as_float(ld4(a.attn, (uint32_t)((m * h + n) * 4)));
        const float v = (res[m * maxrows + rl] + bf_f(W.b2, n)) + resid;
        st4(xo, (uint32_t)((m * h + n) * 4), __float_as_uint(v));
      }
    }
    wg_publish(a, l * E_PER_LAYER + E_FC2);
    STAMP(1 + l * 12 + 11);
    if (l + 1 < L) {
      ws_init(ws, layer_at(a, l + 1).wqkv, h, q0, q1);
      ws_prefetch<P, NTW>(ws, ring);
    } else if (a.has_head) {
      ws_init(ws, a.whead, h, hr0, hr1);
      ws_prefetch<P, NTW>(ws, ring);
    }
  }

  // ================= ln_f + lm_head (slice) + argmax
  if (a.has_head) {
    if (!wg_wait(a, (L - 1) * E_PER_LAYER + E_FC2, producers(h), flag)) goto done;
    STAMP(1 + L * 12 + 0);
    {
      Rows<MM> r;
      rows_load_f32<MM>(r, xout_of(L - 1), M, h);
      rows_ln<MM>(r, h, a.lnf_g, a.lnf_b, a.eps, scr);
      rows_to_xs<MM>(r, h, xs);
    }
    __syncthreads();
    ws_consume<MM, P, NTW>(ws, ring, xs, M, res, maxrows);
    STAMP(1 + L * 12 + 1);
    __syncthreads();
    const int nr = hr1 - hr0, lane = tid & 63, wv = tid >> 6;
    unsigned long long* kscr = reinterpret_cast<unsigned long long*>(scr);  // [8][MM]
#pragma unroll
    for (int m = 0; m < MM; m++) {
      unsigned long long best = 0ull;
      if (m < M) {
        for (int rl = tid; rl < nr; rl += NT) {
          const float v = res[m * maxrows + rl];
          const int col = hr0 + rl;
          if (a.logits) a.logits[(size_t)m * a.ldl + col] = v;
          const unsigned long long key =
              ((unsigned long long)f32_order_key(v) << 32) | (0xFFFFFFFFu - (uint32_t)(col + a.col_offset));
          best = key > best ? key : best;
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
      }
      if (lane == 0) kscr[wv * MM + m] = best;
    }
    __syncthreads();
    if (tid < MM) {
      unsigned long long best = 0ull;
      for (int w = 0; w < NWV; w++) best = kscr[w * MM + tid] > best ? kscr[w * MM + tid] : best;
      __hip_atomic_store((gu64*)(a.wgkeys + (size_t)wg * 4 + tid), best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMP(1 + L * 12 + 2);
  }

  // ================= final ticket: the last workgroup reduces the keys and re-zeroes the state
done:
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add((gu32*)a.fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == (unsigned)(nwg - 1);
  }
  __syncthreads();
  STAMP(1 + L * 12 + 3);
  if (__builtin_amdgcn_readfirstlane(*(volatile int*)flag) == 0) return;
  if (a.has_head && __hip_atomic_load((const gu32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
    const int lane = tid & 63, wv = tid >> 6;
    if (wv < M) {
      unsigned long long best = 0ull;
      for (int w = lane; w < nwg; w += 64) {
        const unsigned long long k =
            __hip_atomic_load((const gu64*)(a.wgkeys + (size_t)w * 4 + wv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        best = k > best ? k : best;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
      }
      if (lane == 0) {
        if (a.keys_in) best = a.keys_in[wv] > best ? a.keys_in[wv] : best;
        if (a.keys_out) a.keys_out[wv] = best;
        if (a.tokens) a.tokens[wv] = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
      }
    }
  }
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int i = tid; i < a.n_ctr_words / 4; i += NT) st16(a.ctr, (uint32_t)i * 16, z);
  for (int i = tid; i < a.n_tick_words; i += NT) st4(a.tick, (uint32_t)i * 4, 0u);
  if (tid == 0) {
    __hip_atomic_store((gu32*)a.err, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32*)a.fin, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int MM>
const void* kernel_ptr() {
  return reinterpret_cast<const void*>(&decode_engine_kernel<MM, 16, true>);
}
const void* kernel_for(int mm) {
  switch (mm) {
    case 1: return kernel_ptr<1>();
    case 2: return kernel_ptr<2>();
    default: return kernel_ptr<4>();
  }
}

}  // namespace

size_t engine_lds_bytes(int mm, int h, int maxrows) {
  const size_t xs = (size_t)mm * 4 * h * 2;
  const size_t res = (size_t)mm * maxrows * 4;
  return ((xs + 15) / 16 * 16) + ((res + 15) / 16 * 16) + 8192;
}

int engine_prepare(int mm, size_t lds, int device) {
  const void* k = kernel_for(mm);
  if (lds > 160 * 1024) return 0;
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, NT, lds) != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    return 0;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
  return cus;  // one workgroup per CU: every workgroup is resident at once
}

void engine_launch(const DeArgs& a, int mm, int grid, size_t lds, hipStream_t s) {
  switch (mm) {
    case 1: decode_engine_kernel<1, 16, true><<<grid, NT, lds, s>>>(a); break;
    case 2: decode_engine_kernel<2, 16, true><<<grid, NT, lds, s>>>(a); break;
    default: decode_engine_kernel<4, 16, true><<<grid, NT, lds, s>>>(a); break;
  }
}
