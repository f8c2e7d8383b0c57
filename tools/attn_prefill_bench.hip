// tools/attn_prefill_bench.hip — prefill attention on the BLOOM prefill shapes: the round-5 kernel
// (attn_prefill_tr_kernel: LDS-DMA K/V, ds_read_b64_tr_b16 V, bf16 P hi + lo) against the round-4 kernel
// (attn_prefill_mfma_kernel: register-staged K, fp16 V^T stores) in one process.  Time = 20 back-to-back
// launches between two HIP events / 20 (a lone launch between events also counts the ~5 us the events add),
// median of 7 such groups.  Numerics: every output element of both kernels against a float64 CPU restatement
// (HF BLOOM attention, modeling_bloom.py:245-310) for head 0 and head nh-1 of row 0 and the last row.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I include tools/attn_prefill_bench.hip
//        -o tools/attn_prefill_bench   (the library's attn_prefill.hip flag; the r4 kernel then also builds in VGPR form)
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include "../distributed_inference_demo_amd/csrc/attn_prefill.hip"
#include <algorithm>

// The round-4 kernel ("r4"), removed from the library in round 5 (fp16 V staging, register-staged K), kept here for the A/B:
// Prefill (S > 1), bf16: MFMA flash attention.  Block = (64-query tile, head, row b), 4 waves x 16
// queries.  Per 64-key tile: K rows and V^T staged in LDS by the block, the NEXT tile's K/V rows
// already in flight to registers while this one computes (the loop was load-latency bound: one
// HBM round trip per 32-key tile, 39 us per bloom-1b1 layer at S = 512); S^T = K.Q^T on
// v_mfma_f32_16x16x32_bf16 (Q fragments in registers, zero-padded past hd), so a lane holds ONE query
// against 16 keys: scale + ALiBi + causal mask + online softmax per lane with two cross-lane steps per
// reduction, and the lane's P values are already the A-operand elements of the P.V MFMAs
// (v_mfma_f32_16x16x32_f16) once V^T is staged in the matching key order (round 4: no P round trip
// through LDS); V is staged as fp16 — exact for bf16 values in fp16's normal range.  P is split into fp16(p) + fp16(p - fp16(p)) and both halves run through the P.V MFMAs,
// so P keeps ~21 bits like the fp32 P of the checker (one fp16 P alone moved bloom-1b1's 512-token
// prefill logits 2.06e-2 off the bf16-mode checker).  q is bf16 (the stage stores q in the
// activation dtype); accumulation and softmax fp32.  The heaviest query tiles (most keys under
// the causal mask) are dispatched first.
// QW waves per block = QW x 16 queries (4: 64-query tiles; 2: 32-query tiles, twice the blocks).
template <int HDP, bool PLO = true, int QW = 4>  // head_dim padded to a multiple of 32 (64, 96, 128); PLO: P hi + lo
__global__ __launch_bounds__(QW * 64) void attn_prefill_mfma_kernel(AttnArgs a) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int QB = QW * 16;            // queries per block
  constexpr int NTH = QW * 64;
  constexpr int KS = HDP / 32;           // k-steps of S = Q.K^T
  constexpr int NT = HDP / 16;           // 16-dim output tiles
  constexpr int KLD = HDP + 8;           // padded K row (bf16 elements)
  constexpr int VLD = KT + 8;            // padded V^T row
  constexpr int CPT = (KT * HDP / 8 + NTH - 1) / NTH;  // 16-B K chunks per thread per tile
  constexpr int VPT = (KT / 4 * HDP / 8 + NTH - 1) / NTH;  // V staging items per thread (4 keys x 8 dims)
  __shared__ __attribute__((aligned(16))) bf16 Ks[KT * KLD];
  __shared__ __attribute__((aligned(16))) _Float16 Vt[HDP * VLD];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  // split-KV (a.pf_tiles > 0): blockIdx.x = (query tile, key split); heaviest query tiles first
  const int nspl = gridDim.x / ((a.S + QB - 1) / QB);
  const int qt = (gridDim.x - 1 - blockIdx.x) / nspl, spl = (gridDim.x - 1 - blockIdx.x) % nspl;
  const int head = blockIdx.y, b = blockIdx.z;
  const int hd = a.head_dim;
  const int past = a.past_dev ? a.past_dev[b] : a.past;
  const int q0 = qt * QB + w * 16;          // first query (within this call) of the wave
  const bf16* qg = (const bf16*)a.q;
  // Q fragments: lane holds Q[q0 + r][ks*32 + 8g .. +8]
  bf16x8 qf[KS];
  {
    const int qrow = min(q0 + r, a.S - 1);
    const bf16* qp = qg + ((size_t)b * a.S + qrow) * a.hidden + head * hd;
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
      const int d = ks * 32 + 8 * g;
      qf[ks] = d < hd ? *reinterpret_cast<const bf16x8*>(qp + d) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const size_t rowbase = ((size_t)(a.slot + b) * a.n_head + head) * a.max_ctx;
  const bf16* kb = (const bf16*)a.k_cache + rowbase * hd;
  const bf16* vb = (const bf16*)a.v_cache + rowbase * hd;
  const float slope = a.slopes[head];
  float m_q = -INFINITY, l_q = 0.f;  // running max / sum of query q0 + r (the 4 lanes r + 16 g agree)
  f32x4 o[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) o[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // keys visible to the block's last query; a split takes key tiles [spl * pf_tiles, + pf_tiles)
  const int kend = past + min(a.S, qt * QB + QB);
  const int kbeg = nspl > 1 ? min(spl * a.pf_tiles * KT, kend) : 0;
  const int kstop = nspl > 1 ? min(kbeg + a.pf_tiles * KT, kend) : kend;
  const int nchunk = hd / 8, nch = KT * nchunk;
  // the padded dims are never staged: zero them once (keeps the MFMA inputs finite)
  if (HDP != 0) {
    for (int c = tid; c < KT * (HDP - hd); c += NTH) {
      const int kr = c / (HDP - hd), d = hd + (c - kr * (HDP - hd));
      Ks[kr * KLD + d] = (bf16)0.f;
      Vt[d * VLD + kr] = (_Float16)0.f;
    }
  }
  // V^T row d keeps its 8-key chunks XOR-swizzled by (d >> 3): the transposing element stores of a
  // wave (lanes = 8-dim slices of a few keys) then spread over the LDS banks instead of two
  auto vsw = [](int d, int key) { return d * VLD + ((((key >> 3) ^ (d >> 3)) & 7) << 3) + (key & 7); };
  // V^T keys are stored in the order the P fragments come out of the S^T accumulators: in each 32-key block,
  // key 16 h + 4 g + j sits at 8 g + 4 h + j, so lane group g's 8 k-elements of a P.V step are contiguous
  auto kperm = [](int k) { return (k & ~31) | (((k >> 2) & 3) << 3) | (((k >> 4) & 1) << 2) | (k & 3); };
  // V is staged by (4 keys x 8 dims) items: one 8-B LDS store per dim writes 4 keys of V^T
  // (VPT items per thread; KT/4 * hd/8 <= 256 items)
  const int nvi = (KT / 4) * nchunk;
  int vq[VPT], vdc[VPT];
#pragma unroll
  for (int v = 0; v < VPT; v++) {
    const int it = min(tid + v * NTH, nvi - 1);
    vq[v] = it / nchunk;
    vdc[v] = (it % nchunk) * 8;
  }
  // one register stage: tile k0 + KT is in flight while tile k0 computes (a second stage, tile k0 + 2 KT,
  // measured no faster: profiles/r03_attn_prefill_split.txt)
  bf16x8 kreg[CPT], vreg[VPT][4];
  auto gload = [&](int k0, int lim) {  // clamped to key lim: loads past it re-read that key
#pragma unroll
    for (int i = 0; i < CPT; i++) {
      const int c = min(tid + i * NTH, nch - 1);
      const int kr = c / nchunk, dc = (c - kr * nchunk) * 8;
      const int key = min(k0 + kr, lim);
      kreg[i] = *reinterpret_cast<const bf16x8*>(kb + (size_t)key * hd + dc);
    }
#pragma unroll
    for (int v = 0; v < VPT; v++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int key = min(k0 + vq[v] * 4 + i, lim);
        vreg[v][i] = *reinterpret_cast<const bf16x8*>(vb + (size_t)key * hd + vdc[v]);
      }
  };
  // The first tile is requested at the split's nominal start, clamped to the cache rather than to the
  // context, so it does not wait for past_len: keys past the context are masked (p = 0) and their V is
  // staged as 0 (below).  An empty split drops it.
  gload(nspl > 1 ? min(spl * a.pf_tiles * KT, a.max_ctx - 1) : 0, a.max_ctx - 1);
  for (int k0 = kbeg; k0 < kstop; k0 += KT) {
    __syncthreads();  // previous tile's LDS reads are done
#pragma unroll
    for (int i = 0; i < CPT; i++) {
      const int c = tid + i * NTH;
      if (c < nch) {
        const int kr = c / nchunk, dc = (c - kr * nchunk) * 8;
        *reinterpret_cast<bf16x8*>(&Ks[kr * KLD + dc]) = kreg[i];
      }
    }
#pragma unroll
    for (int v = 0; v < VPT; v++) {
      if (tid + v * NTH < nvi) {
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        // keys past the split's end are staged as 0: their p is 0, but a stale cache row there (an earlier
        // request's, past this one's context) could hold a value outside fp16's range, and 0 * inf is NaN
        const int kv0 = k0 + vq[v] * 4;
        const bool ok0 = kv0 < kstop, ok1 = kv0 + 1 < kstop, ok2 = kv0 + 2 < kstop, ok3 = kv0 + 3 < kstop;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const f16x4 v4 = {ok0 ? (_Float16)(float)vreg[v][0][j] : (_Float16)0.f, ok1 ? (_Float16)(float)vreg[v][1][j] : (_Float16)0.f,
                            ok2 ? (_Float16)(float)vreg[v][2][j] : (_Float16)0.f, ok3 ? (_Float16)(float)vreg[v][3][j] : (_Float16)0.f};
          *reinterpret_cast<f16x4*>(&Vt[vsw(vdc[v] + j, kperm(vq[v] * 4))]) = v4;
        }
      }
    }
    __syncthreads();
    if (k0 + KT < kstop) gload(k0 + KT, kend - 1);  // next tile in flight while this one computes
    // S^T tiles: four 16-key tiles, K as the A operand and Q as B, so lane (r, g) holds query q0 + r against keys
    // t*16 + 4g + i: a query's softmax statistics need two cross-lane steps (xor 16, xor 32) instead of four DPP
    // steps per row, and its P values feed the P.V A operand straight from registers (no LDS round trip)
    f32x4 sacc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
      sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ks++) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[(t * 16 + r) * KLD + ks * 32 + 8 * g]);
        sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], sacc[t], 0, 0, 0);
      }
    }
    // scale, ALiBi, causal mask
    const int qpos = past + q0 + r;
    float sv[4][4], rmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int kpos = k0 + t * 16 + 4 * g + i;
        const float v = (kpos <= qpos && kpos < kstop) ? slope * (float)kpos + a.inv_norm * sacc[t][i] : -INFINITY;
        sv[t][i] = v;
        rmax = fmaxf(rmax, v);
      }
    rmax = fmaxf(rmax, __shfl_xor(rmax, 16, 64));
    rmax = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
    const float m_new = fmaxf(m_q, rmax);
    // queries whose keys are all masked so far keep m = -inf; exp(-inf - -inf) guarded
    const float scale_q = m_new == -INFINITY ? 1.f : __expf(m_q - m_new);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const float p = m_new == -INFINITY ? 0.f : __expf(sv[t][i] - m_new);
        sv[t][i] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_q = l_q * scale_q + rs;
    m_q = m_new;
    // the output accumulators hold queries 4g + i: their scales come from lanes 4g + i
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float sc = __shfl(scale_q, 4 * g + i, 64);
#pragma unroll
      for (int t = 0; t < NT; t++) o[t][i] *= sc;
    }
    // P fragments of the two 32-key steps: keys 32 kb + 16 h + 4 g + j (h, j < 2, 4) = tiles 2 kb + h, element j;
    // P = fp16(p) + fp16(p - fp16(p)) (~21 bits)
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
    f16x8 pf[2], pl[2];
#pragma unroll
    for (int kb = 0; kb < 2; kb++)
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const float p = sv[2 * kb + (e >> 2)][e & 3];
        const _Float16 hi = (_Float16)p;
        pf[kb][e] = hi;
        pl[kb][e] = (_Float16)(p - (float)hi);
      }
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const f16x8 vf0 = *reinterpret_cast<const f16x8*>(&Vt[vsw(t * 16 + r, 8 * g)]);
      const f16x8 vf1 = *reinterpret_cast<const f16x8*>(&Vt[vsw(t * 16 + r, 32 + 8 * g)]);
      o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf[0], vf0, o[t], 0, 0, 0);
      o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf[1], vf1, o[t], 0, 0, 0);
      if constexpr (PLO) {
        o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl[0], vf0, o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl[1], vf1, o[t], 0, 0, 0);
      }
    }
  }
  // the statistics of the accumulator rows (queries q0 + 4g + i)
  float m_run[4], l_run[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    m_run[i] = __shfl(m_q, 4 * g + i, 64);
    l_run[i] = __shfl(l_q, 4 * g + i, 64);
  }
  if (nspl > 1) {
    // split partial (running max, sum, unnormalised context) of the block's 64 queries, write-through:
    // record [m, l, -, -, o[0..hd)] per (split, query); the block drawing the last ticket of its (row,
    // head, query tile) merges the splits in split order
    const int rs = hd + 4;
    const size_t item = ((size_t)(b * a.n_head + head) * ((a.S + QB - 1) / QB) + qt);
    const __amdgpu_buffer_rsrc_t rp = attn_rsrc(a.pf_ws + item * nspl * QB * rs);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int ql = w * 16 + 4 * g + i;
      const uint32_t rec = (uint32_t)((spl * QB + ql) * rs) * 4;
      if (r == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m_run[i]), rp, rec, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l_run[i]), rp, rec + 4, 0, 16);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const int d = t * 16 + r;
        if (d < hd) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[t][i]), rp, rec + (4 + d) * 4, 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int last;
    __syncthreads();
    if (tid == 0) {
      typedef __attribute__((address_space(1))) unsigned gu32;
      const unsigned old = __hip_atomic_fetch_add((gu32*)(a.pf_tickets + item), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == (unsigned)(nspl - 1);
      if (last) __hip_atomic_store((gu32*)(a.pf_tickets + item), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    // merge: 4 threads per query, each a quarter of its 4-dim chunks; splits in groups of 4 whose loads
    // are all issued before use (indices clamped, surplus splits weighted 0), online max across groups
    const int ql = tid >> 2, j = tid & 3, nc = hd / 4;
    constexpr int G = 4, NC = HDP / 16;  // chunks per thread: ceil(HDP/4 / 4)
    float M = -INFINITY, Lsum = 0.f;
    f32x4 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < nspl; s0 += G) {
      float mg[G], lg[G];
      f32x4 og[G][NC];
#pragma unroll
      for (int u = 0; u < G; u++) {
        const uint32_t rec = (uint32_t)((min(s0 + u, nspl - 1) * QB + ql) * rs) * 4;
        mg[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, rec, 0, 16));
        lg[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, rec + 4, 0, 16));
#pragma unroll
        for (int c = 0; c < NC; c++)
          og[u][c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rp, rec + (4 + 4 * min(j + 4 * c, nc - 1)) * 4, 0, 16));
      }
      float mn = M;
#pragma unroll
      for (int u = 0; u < G; u++)
        if (s0 + u < nspl) mn = fmaxf(mn, mg[u]);
      const float sc = M == -INFINITY ? 0.f : __expf(M - mn);  // mn is finite: split 0 holds key 0
      Lsum *= sc;
#pragma unroll
      for (int c = 0; c < NC; c++) acc[c] *= sc;
#pragma unroll
      for (int u = 0; u < G; u++) {
        // a split past the query's keys (m = -inf) or past nspl weighs 0
        const float wu = (s0 + u < nspl && mg[u] != -INFINITY) ? __expf(mg[u] - mn) : 0.f;
        Lsum += wu * lg[u];
#pragma unroll
        for (int c = 0; c < NC; c++) acc[c] += wu * og[u][c];
      }
      M = mn;
    }
    const int q = qt * QB + ql;
    if (q < a.S) {
      const float inv = 1.f / Lsum;
      bf16* op = (bf16*)a.ctx_out + ((size_t)b * a.S + q) * a.hidden + head * hd;
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const int ch = j + 4 * c;
        if (ch < nc) {
          bf16 v4[4] = {(bf16)(acc[c][0] * inv), (bf16)(acc[c][1] * inv), (bf16)(acc[c][2] * inv), (bf16)(acc[c][3] * inv)};
          *reinterpret_cast<uint2*>(op + 4 * ch) = *reinterpret_cast<const uint2*>(v4);
        }
      }
    }
    return;
  }
  // write ctx rows (q = q0 + 4g + i, dim = t*16 + r)
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int q = q0 + 4 * g + i;
    if (q >= a.S) continue;
    const float inv = 1.0f / l_run[i];
    bf16* op = (bf16*)a.ctx_out + ((size_t)b * a.S + q) * a.hidden + head * hd;
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const int d = t * 16 + r;
      if (d < hd) op[d] = (bf16)(o[t][i] * inv);
    }
  }
}

// split-KV: a query tile's keys over ceil(tiles / pf_tiles) blocks when the grid would leave CUs idle and the
// partials fit (the longest query tile otherwise walks every key tile alone).  QW waves per block (QW x 16 queries).
template <int QW>
static void attn_prefill_mfma_launch(const AttnArgs& a, hipStream_t s) {
  constexpr int QB = QW * 16;
  const int nqt = (a.S + QB - 1) / QB;
  const int ktiles = (a.pf_past_max + a.S + 63) / 64;  // the last query tile's, longest row
  int nspl = 1;
  if (a.pf_tiles > 0 && a.pf_ws && a.pf_tickets && (long)nqt * a.n_head * a.B < 256 * 4 / QW && ktiles > a.pf_tiles) {
    nspl = (ktiles + a.pf_tiles - 1) / a.pf_tiles;
    const size_t need = (size_t)a.B * a.n_head * nqt * nspl * QB * (a.head_dim + 4);
    if (need > a.pf_cap || (long)a.B * a.n_head * nqt > a.pf_ntickets) nspl = 1;
  }
  dim3 g(nqt * nspl, a.n_head, a.B);
  const int hdp = (a.head_dim + 31) / 32 * 32;
  if (hdp <= 64) attn_prefill_mfma_kernel<64, true, QW><<<g, QW * 64, 0, s>>>(a);
  else if (hdp <= 96) attn_prefill_mfma_kernel<96, true, QW><<<g, QW * 64, 0, s>>>(a);
  else attn_prefill_mfma_kernel<128, true, QW><<<g, QW * 64, 0, s>>>(a);
}


#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12;
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * scale);
  }
}

static float bf(bf16 v) { return (float)v; }

int main(int argc, char** argv) {
  struct Sh { const char* name; int B, S, past, nh, hd; } shapes[] = {
      {"7b1 S512", 1, 512, 0, 32, 128}, {"3b S512", 1, 512, 0, 32, 80}, {"1b1 S512", 1, 512, 0, 16, 96},
      {"560m S512", 1, 512, 0, 16, 64}, {"7b1 B2 S512", 2, 512, 0, 32, 128}, {"1b1 S128", 1, 128, 0, 16, 96},
      {"1b1 S256+past768", 1, 256, 768, 16, 96}, {"7b1 B4 S1024", 4, 1024, 0, 32, 128},
      {"7b1 B1 S16x16", 16, 16, 0, 32, 128}};
  const int max_ctx = 2048;
  bf16 *q, *kc, *vc, *ctx; float *slopes, *ws; unsigned* tick; int* pastd;
  const size_t qn = (size_t)16 * 1024 * 4096;
  const size_t kvn = (size_t)16 * 32 * max_ctx * 128;
  CK(hipMalloc(&q, qn * 2)); CK(hipMalloc(&ctx, qn * 2));
  CK(hipMalloc(&kc, kvn * 2)); CK(hipMalloc(&vc, kvn * 2));
  CK(hipMalloc(&slopes, 64 * 4)); CK(hipMalloc(&pastd, 64 * 4));
  const size_t cap = (size_t)480 * 128 * 128;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  fill_rand<<<4096, 256>>>(q, qn, 1, 2.f); fill_rand<<<4096, 256>>>(kc, kvn, 2, 2.f); fill_rand<<<4096, 256>>>(vc, kvn, 3, 2.f);
  std::vector<float> hs(64);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    for (int i = 0; i < sh.nh; i++) hs[i] = powf(2.f, -8.f * (i + 1) / sh.nh);
    CK(hipMemcpy(slopes, hs.data(), 64 * 4, hipMemcpyHostToDevice));
    std::vector<int> hp(64, sh.past);
    CK(hipMemcpy(pastd, hp.data(), 64 * 4, hipMemcpyHostToDevice));
    AttnArgs a{};
    a.q = q; a.k_cache = kc; a.v_cache = vc; a.ctx_out = ctx; a.slopes = slopes;
    a.B = sh.B; a.S = sh.S; a.slot = 0; a.past_dev = pastd; a.past = sh.past; a.n_head = sh.nh; a.head_dim = sh.hd;
    a.max_ctx = max_ctx; a.hidden = sh.nh * sh.hd; a.inv_norm = 1.f / sqrtf((float)sh.hd);
    a.pf_ws = ws; a.pf_cap = cap; a.pf_tickets = tick; a.pf_ntickets = 4096; a.pf_past_max = sh.past; a.pf_tiles = 4;
    const size_t on = (size_t)sh.B * sh.S * a.hidden;
    // float64 reference for (row, head) pairs
    std::vector<bf16> hq((size_t)sh.B * sh.S * a.hidden), hk, hv;
    CK(hipMemcpy(hq.data(), q, hq.size() * 2, hipMemcpyDeviceToHost));
    const int rows_chk[2] = {0, sh.B - 1}, heads_chk[2] = {0, sh.nh - 1};
    std::vector<std::vector<double>> ref;
    for (int bi : rows_chk)
      for (int hh : heads_chk) {
        const size_t base = ((size_t)bi * sh.nh + hh) * max_ctx * sh.hd;
        std::vector<bf16> K((size_t)(sh.past + sh.S) * sh.hd), Vv(K.size());
        CK(hipMemcpy(K.data(), kc + base, K.size() * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(Vv.data(), vc + base, Vv.size() * 2, hipMemcpyDeviceToHost));
        std::vector<double> out((size_t)sh.S * sh.hd);
        for (int t = 0; t < sh.S; t++) {
          const int nk = sh.past + t + 1;
          std::vector<double> sc(nk);
          double mx = -1e300;
          for (int j = 0; j < nk; j++) {
            double d = 0;
            for (int e = 0; e < sh.hd; e++) d += (double)bf(hq[((size_t)bi * sh.S + t) * a.hidden + hh * sh.hd + e]) * bf(K[(size_t)j * sh.hd + e]);
            sc[j] = (double)hs[hh] * j + (double)a.inv_norm * d;
            mx = std::max(mx, sc[j]);
          }
          double sum = 0;
          for (int j = 0; j < nk; j++) { sc[j] = exp(sc[j] - mx); sum += sc[j]; }
          for (int e = 0; e < sh.hd; e++) {
            double o = 0;
            for (int j = 0; j < nk; j++) o += sc[j] * bf(Vv[(size_t)j * sh.hd + e]);
            out[(size_t)t * sh.hd + e] = o / sum;
          }
        }
        ref.push_back(out);
      }
    std::vector<bf16> ho(on);
    // variants: (stages, key tiles per split, split when units < max_units); the last is the round-4 kernel
    // (round 5, second pass: kg / qg = -1 is the library's choice by shape; qg 2 = two query groups per wave)
    // (round 6 also ran a software-pipelined loop here, sp = 1: profiles/r06_attn_prefill_sp_ab.txt, not kept)
    struct Vr { int nstg, pt, mu, kg, qg; } vars[] = {
        {2, 4, 256, -1, -1}, {2, 4, 256, 1, 1}, {3, 4, 256, 1, 1}, {2, 2, 512, 1, 1}, {2, 8, 256, 1, 1},
        {2, 4, 256, 1, 2}, {2, 4, 256, 2, 1}};
    for (int kern = 0; kern < (int)(sizeof(vars) / sizeof(vars[0])); kern++) {
      const Vr vr = vars[kern];
      auto launch = [&]() { if (vr.nstg) attn_prefill_tr_launch(a, 0, vr.nstg, vr.pt, vr.mu, vr.kg, vr.qg); else attn_prefill_mfma_launch<4>(a, 0); };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ho.data(), ctx, on * 2, hipMemcpyDeviceToHost));
      double md = 0, mref = 0;
      int k = 0;
      for (int bi : rows_chk)
        for (int hh : heads_chk) {
          for (int t = 0; t < sh.S; t++)
            for (int e = 0; e < sh.hd; e++) {
              const double r0 = ref[k][(size_t)t * sh.hd + e];
              const double g0 = bf(ho[((size_t)bi * sh.S + t) * a.hidden + hh * sh.hd + e]);
              md = std::max(md, fabs(g0 - r0) / (fabs(r0) * 0x1p-8 + 1e-3));
              mref = std::max(mref, fabs(r0));
            }
          k++;
        }
      std::vector<float> t;
      for (int it = 0; it < 7; it++) {
        CK(hipEventRecord(e0));
        for (int rep = 0; rep < 20; rep++) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3f / 20);
      }
      std::sort(t.begin(), t.end());
      double flops = 0;
      for (int tq = 0; tq < sh.S; tq++) flops += 4.0 * (sh.past + tq + 1) * sh.hd;
      flops *= (double)sh.B * sh.nh;
      char nm[32];
      if (vr.nstg) snprintf(nm, sizeof nm, "s%d p%d u%d g%d q%d", vr.nstg, vr.pt, vr.mu, vr.kg, vr.qg);
      else snprintf(nm, sizeof nm, "r4");
      printf("%-18s B=%d S=%4d past=%4d nh=%2d hd=%3d  %-20s %7.2f us/launch (min %7.2f)  %6.1f TFLOP/s  err/(ulp+1e-3) max %.3f\n",
             sh.name, sh.B, sh.S, sh.past, sh.nh, sh.hd, nm, t[t.size() / 2], t[0],
             flops / (t[t.size() / 2] * 1e-6) / 1e12, md);
    }
  }
  return 0;
}
