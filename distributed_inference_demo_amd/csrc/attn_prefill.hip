// attn_prefill.hip — prefill (S > 1) bf16 attention of one BLOOM stage, gfx950 (MI355X).  Its own translation unit:
// it is compiled with -mllvm -amdgpu-mfma-vgpr-form=1 (build.py), so the P.V accumulators stay in VGPRs and the
// per-tile rescale is plain VALU (in the AGPR form the compiler moved all 32 accumulators AGPR -> VGPR -> AGPR every
// key tile); the other kernels keep the default form (the flag makes the rows GEMVs spill).
// Math restated from HF BLOOM BloomAttention.forward (modeling_bloom.py:245-310): scores = alibi + q.k / sqrt(hd),
// causal mask, fp32 softmax, context = P.V -- what the reference's ONNX sub-models execute (inference.cpp:207-215).
#include "common.h"
#include "kernels.h"

namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
template <int V> struct IntC { static constexpr int value = V; };
}  // namespace

// Prefill (S > 1), bf16, round 5: MFMA flash attention on LDS-DMA-staged K/V tiles.
// Block = 64 queries (4 waves x 16) of one (row, head) [x one key split]; per 64-key tile:
//  * K and V arrive by LDS-DMA (buffer_load ... lds: no VGPR staging, no ds_write, no conversion) into an
//    NSTG-deep ring, tile t + NSTG - 1 in flight while tile t computes, one raw s_barrier per tile;
//  * LDS image = the guide's layout (b) for [64 rows][128 x 16-bit] tiles (cdna_hip_programming.md T10): byte
//    offset 256 row + 16 (chunk ^ ((row & 3) << 2 | (row >> 2) & 3)); the XOR is applied on the global side
//    (the lane filling LDS chunk c of a row fetches logical chunk c ^ swz(row)), so the DMA stays contiguous;
//  * S^T = K.Q^T on v_mfma_f32_16x16x32_bf16 (K rows by ds_read_b128, Q fragments in registers, zero past
//    head_dim): lane (r, g) holds query r against 16 keys -- softmax statistics in two cross-lane steps, and
//    the lane's P values are already the A operand of P.V;
//  * P.V reads V straight from its row-major image with ds_read_b64_tr_b16 (the hardware transpose: lane i of
//    a 16-lane group receives column i of 4 rows), no transposing stores; the rows each group reads are the
//    keys its P values belong to, so A and B agree key for key.  Key rows of A are permuted (group g of a
//    16-key subtile holds keys 4 perm(g) .. + 3, perm = 0, 2, 1, 3) so the two groups of a 32-lane half
//    read row blocks 8 apart: conflict-free transposed reads;
//  * V stays bf16 (no fp16 range limit, any finite cache value is exact); P = bf16(p) + bf16(p - bf16(p))
//    runs through the P.V MFMAs as two operands (~16 significant bits of P, the rest below the bf16 rounding
//    of the context: tools/parity_study.py emul_bf16), accumulation and softmax fp32;
//  * head_dim <= 128 padded to 128 in LDS (row r of the cache is hd x 2 bytes; lanes past hd re-read the
//    row's last chunk, finite, multiplied by Q's zero dims or landing in discarded output columns); the
//    k-steps and output tiles past hd are skipped (wave-uniform bounds);
//  * blocks of one (row, head) share an XCD (blocks b and b + 8 do under round-robin dispatch: speed only)
//    when the pair count is a multiple of 8, so their K/V re-reads hit that XCD's L2; the heaviest units
//    (most keys under the causal mask) are dispatched first;
//  * split-KV (a.pf_tiles > 0, small grids): as before, (m, l, unnormalised context) records write-through
//    and the last-arriving block merges in split order.
// Keys past a block's context are masked (p = 0); their V rows are finite (the cache is zeroed at init and
// holds only finite bf16 values), and rows past max_ctx read 0 through the bounded buffer descriptor.
// Diagnostic builds only (tools/attn_prefill_bench.hip defines ATTN_STAMPS): wave 0 of each block records s_memtime
// (shader clock) at phase boundaries of its first 16 key tiles into LDS, written out at the end.
#ifdef ATTN_STAMPS
__device__ unsigned long long g_attn_stamps[4096 * 17 * 8];
#define ATTN_STAMP(it, ph) do { __builtin_amdgcn_sched_barrier(0); \
    if (threadIdx.x == 0 && (it) < 16) st_lds[(it) * 8 + (ph)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define ATTN_STAMP(it, ph) do {} while (0)
#endif
__device__ __forceinline__ int attn_tr_off(int row, int ch) {  // byte offset in a [64][128] bf16 tile image
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// Cross-lane max / sum with the partner lane l ^ 16 or l ^ 32 by v_permlane16/32_swap (VALU, no LDS round trip):
// with both operands x, one output holds x[l] and the other x[l ^ 16] (or ^ 32) on every lane (tools/probe/
// permlane_probe.hip), and both lanes of a pair combine them in the same order.
__device__ __forceinline__ float attn_xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float attn_xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float attn_xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float attn_xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// HDE: head_dim rounded up to 64 / 96 / 128 -- the k-steps of Q.K^T (HDE / 32) and the 16-dim output tiles (HDE / 16)
// are compile-time, so every LDS read of a tile is issued before the MFMAs that wait on it (runtime-uniform guards in
// the unrolled loops serialised read -> wait -> MFMA: tools/attn_stamps.hip, profiles/r05_attn_stamps.txt).
// P.V runs as O^T = V^T . P^T (A = the transposed V reads, B = the P registers): a lane's accumulators are dims
// 4g .. 4g + 3 of ITS query r, so the per-query rescale and the final 1 / l are lane-local.
// KG key groups: KG x 4 waves per block; group kg (waves 4 kg .. 4 kg + 3, the same 64 queries) takes the block's key
// tiles kg, kg + KG, ... with its own LDS ring, and the groups' (m, l, o) meet in LDS at the end -- a split of the keys
// with no global partials and no ticket, and two waves per SIMD.  KG = 2 halves the serial tile chain of the longest
// (causal) query tiles.
// QG query groups per wave (KG = 1, no key split): a wave takes 16 QG queries, so every K fragment and every
// transposed V read of a tile feeds QG MFMAs -- half the LDS reads per MFMA at QG = 2 (128-query blocks, for grids
// with blocks to spare).
template <int NSTG, int HDE, int KG, int QG = 1>
__global__ __launch_bounds__(256 * KG) void attn_prefill_tr_kernel(AttnArgs a, int nspl, int U, int xcd_group) {
  static_assert(QG == 1 || KG == 1, "query groups with one key group");
  constexpr int KT = 64, QB = 64 * QG, TILEB = KT * 256;
  constexpr int KSE = HDE / 32, NTE = HDE / 16;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((address_space(3))) void lds_void;
  __shared__ __attribute__((aligned(16))) unsigned char smem[KG * NSTG * 2 * TILEB];
#ifdef ATTN_STAMPS
  __shared__ unsigned long long st_lds[17 * 8];
  if (threadIdx.x == 0) st_lds[16 * 8] = __builtin_amdgcn_s_memtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int kg = KG > 1 ? (tid >> 8) : 0, w = (tid >> 6) & 3;  // key group, wave within the group (query sub-tile)
  const int P = a.B * a.n_head;
  int pair, u;
  if (xcd_group) {  // P % 8 == 0: pair = 8 j' + (id % 8), every unit of a pair on one XCD
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, pg = P >> 3;
    pair = (j % pg) * 8 + xcd;
    u = U - 1 - j / pg;
  } else {
    pair = blockIdx.x % P;
    u = U - 1 - blockIdx.x / P;
  }
  const int qt = u / nspl, spl = u - qt * nspl;
  const int b = pair / a.n_head, head = pair - b * a.n_head;
  const int hd = a.head_dim, nch = hd >> 3;
  const size_t rowbase = ((size_t)(a.slot + b) * a.n_head + head) * a.max_ctx;
  const int cbytes = a.max_ctx * hd * 2;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>((const bf16*)a.k_cache + rowbase * hd), (short)0, cbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>((const bf16*)a.v_cache + rowbase * hd), (short)0, cbytes, 0x00020000);
  // DMA: wave w fills pieces 4w .. 4w + 3 (1 KB = 4 rows each) of the K and the V tile; lane l of piece pc
  // writes LDS chunk l & 15 of row 4 pc + (l >> 4) and fetches that row's logical chunk (l & 15) ^ swz(row)
  uint32_t voff[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int pc = 4 * w + i, row = 4 * pc + (lane >> 4);
    const int x = (lane & 15) ^ (((lane >> 4) << 2) | (pc & 3));
    voff[i] = (uint32_t)(row * hd * 2 + min(x, nch - 1) * 16);
  }
  auto Ks = [&](int st) { return smem + (kg * NSTG + st) * 2 * TILEB; };
  auto Vs = [&](int st) { return smem + (kg * NSTG + st) * 2 * TILEB + TILEB; };
  auto issue = [&](int st, int k0) {  // rows past max_ctx read 0
    const int so = k0 * hd * 2;
#pragma unroll
    for (int i = 0; i < 4; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(Ks(st) + (4 * w + i) * 1024), 16, voff[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void*)(Vs(st) + (4 * w + i) * 1024), 16, voff[i], so, 0, 0);
  };
  // Q first (older than the DMAs in the wave's vmcnt order, so its wait leaves the tiles in flight)
  const int q0 = qt * QB + w * 16 * QG;  // the wave's first query; group j: queries q0 + 16 j + r
  bf16x8 qf[QG][KSE];
#pragma unroll
  for (int j = 0; j < QG; j++) {
    const int qrow = min(q0 + 16 * j + r, a.S - 1);
    const bf16* qp = (const bf16*)a.q + ((size_t)b * a.S + qrow) * a.hidden + head * hd;
#pragma unroll
    for (int ks = 0; ks < KSE; ks++) {
      const int d = ks * 32 + 8 * g;
      qf[j][ks] = d < hd ? *reinterpret_cast<const bf16x8*>(qp + d) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // the first tiles are requested at the split's nominal start before past_len is read (it may come from
  // device memory): a split that turns out empty never reads them
  const int knom = nspl > 1 ? spl * a.pf_tiles * KT : 0;
#pragma unroll
  for (int i = 0; i < NSTG - 1; i++) issue(i, knom + (i * KG + kg) * KT);
  const int past = a.past_dev ? a.past_dev[b] : a.past;
  const float slope = a.slopes[head];
  const int kend = past + min(a.S, qt * QB + QB);  // keys visible to the block's last query
  const int kbeg = min(knom, kend);
  const int kstop = nspl > 1 ? min(kbeg + a.pf_tiles * KT, kend) : kend;
  const int ntile = (kstop - kbeg + KT - 1) / KT;
  const int nit = (ntile + KG - 1) / KG;  // loop trips (every group runs them all: the barriers are block-wide)
  // running max / sum of query q0 + 16 j + r (every lane of the query agrees)
  float m_q[QG], l_q[QG];
  f32x4 o[QG][NTE];  // o[j][t][i] = unnormalised context of query q0 + 16 j + r, dim 16 t + 4 g + i
#pragma unroll
  for (int j = 0; j < QG; j++) {
    m_q[j] = -INFINITY;
    l_q[j] = 0.f;
#pragma unroll
    for (int t = 0; t < NTE; t++) o[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int pg4 = ((g & 1) << 1) | (g >> 1);  // perm(g): this lane group's 4-key block in every 16-key subtile
  const int arow = ((((r >> 2) & 1) << 1) | (r >> 3)) * 4 + (r & 3);  // key (within a subtile) of A row r
  const int qpos = past + q0 + r;  // group j: qpos + 16 j
  const int qq = r >> 2, pp = r & 3;
  // S^T = K.Q^T of the tile in stage st: every K fragment of the tile read, then the MFMAs
  auto kq = [&](int st, f32x4 (&sacc)[QG][4]) {
    const unsigned char* ks_ = Ks(st);
    bf16x8 kf[4][KSE];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int ks = 0; ks < KSE; ks++)
        kf[t][ks] = *reinterpret_cast<const bf16x8*>(ks_ + attn_tr_off(t * 16 + arow, ks * 4 + g));
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int j = 0; j < QG; j++) {
        sacc[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KSE; ks++)
          sacc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][ks], qf[j][ks], sacc[j][t], 0, 0, 0);
      }
  };
  // scale, ALiBi, causal mask, online softmax of the tile at k0 (scores in sacc), then O += P.V from stage st
  auto softmax_pv = [&](int it, int st, int k0, const f32x4 (&sacc)[QG][4]) {
    // sacc[t][i] is key k0 + 16 t + 4 perm(g) + i against query q0 + r; the mask only on the tiles that cross the
    // wave's diagonal or the split's end (wave-uniform test)
    float sv[QG][4][4];
    const float abase = slope * (float)(k0 + 4 * pg4);
    const bool full = k0 + KT - 1 <= past + q0 && k0 + KT <= kstop;  // (group 0's first query is the earliest)
#pragma unroll
    for (int j = 0; j < QG; j++)
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) sv[j][t][i] = fmaf(a.inv_norm, sacc[j][t][i], fmaf(slope, (float)(t * 16 + i), abase));
    if (!full) {
#pragma unroll
      for (int j = 0; j < QG; j++)
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int kpos = k0 + t * 16 + 4 * pg4 + i;
            sv[j][t][i] = (kpos <= qpos + 16 * j && kpos < kstop) ? sv[j][t][i] : -INFINITY;
          }
    }
    float rmax[QG];
#pragma unroll
    for (int j = 0; j < QG; j++) {
      rmax[j] = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) rmax[j] = fmaxf(rmax[j], sv[j][t][i]);
    }
    ATTN_STAMP(it, 4);
#pragma unroll
    for (int j = 0; j < QG; j++) {
      rmax[j] = attn_xmax32(attn_xmax16(rmax[j]));
      const float m_new = fmaxf(m_q[j], rmax[j]);
      const float scale_q = m_new == -INFINITY ? 1.f : __expf(m_q[j] - m_new);
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float p = m_new == -INFINITY ? 0.f : __expf(sv[j][t][i] - m_new);
          sv[j][t][i] = p;
          rs += p;
        }
      rs = attn_xsum32(attn_xsum16(rs));
      l_q[j] = l_q[j] * scale_q + rs;
      m_q[j] = m_new;
#pragma unroll
      for (int t = 0; t < NTE; t++) o[j][t] *= scale_q;
    }
    ATTN_STAMP(it, 5);
    // P^T (B operand of step kb): element e = key 32 kb + 16 (e >> 2) + 4 perm(g) + (e & 3) of query r; hi + lo
    bf16x8 ph[QG][2], pl[QG][2];
#pragma unroll
    for (int j = 0; j < QG; j++)
#pragma unroll
      for (int kb = 0; kb < 2; kb++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const float p = sv[j][2 * kb + (e >> 2)][e & 3];
          const bf16 hi = (bf16)p;
          ph[j][kb][e] = hi;
          pl[j][kb][e] = (bf16)(p - (float)hi);
        }
    ATTN_STAMP(it, 6);
    // V^T fragments by transposed reads: lane 4q + p of group g addresses row (32 kb + 16 h + 4 perm(g) + q), columns
    // 16 t + 4 p .. + 3, and lane r receives column 16 t + r of those 4 rows
    const unsigned char* vs_ = Vs(st);
#pragma unroll
    for (int t = 0; t < NTE; t++)
#pragma unroll
      for (int kb = 0; kb < 2; kb++) {
        const int rw0 = 32 * kb + 4 * pg4 + qq;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(vs_ + attn_tr_off(rw0, 2 * t + (pp >> 1)) + 8 * (pp & 1)));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(vs_ + attn_tr_off(rw0 + 16, 2 * t + (pp >> 1)) + 8 * (pp & 1)));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
#pragma unroll
        for (int j = 0; j < QG; j++) {
          o[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, ph[j][kb], o[j][t], 0, 0, 0);
          o[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pl[j][kb], o[j][t], 0, 0, 0);
        }
      }
  };
  // (Round 6 measured a software-pipelined form of this loop -- three LDS stages, tile it + 1's K.Q^T MFMAs issued
  // ahead of tile it's softmax -- at 0.95-1.01x on the BLOOM prefill shapes and 0.7x with two query groups, which
  // then lose their second block per CU: profiles/r06_attn_prefill_sp_ab.txt.  Not kept.)
  for (int it = 0; it < nit; it++) {
    const int st = it % NSTG, ti = it * KG + kg, k0 = kbeg + ti * KT;
    ATTN_STAMP(it, 0);
    // this wave's DMA of tile it retired (the NSTG - 2 younger tiles stay in flight) -> barrier: every wave's
    // pieces landed and every wave is done reading the stage the next DMA overwrites
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NSTG - 2)) : "memory");
    ATTN_STAMP(it, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    ATTN_STAMP(it, 2);
    // always issue (past the end: a clamped re-read into a free stage) so the counted waits stay exact
    issue((it + NSTG - 1) % NSTG, min(k0 + (NSTG - 1) * KG * KT, a.max_ctx));
    ATTN_STAMP(it, 3);
    if (ti >= ntile) continue;  // this group's share ran out (wave-uniform); it still meets the barriers
    f32x4 sacc[QG][4];
    kq(st, sacc);
    softmax_pv(it, st, k0, sacc);
  }
  // the clamped DMAs still in flight land before the LDS is reused or the block exits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (KG == 2) {
    // group 1 hands (m, l, o) to group 0 through LDS (group 1's ring), lane for lane: the same layout on both sides
    __syncthreads();
    float* xm = reinterpret_cast<float*>(smem + NSTG * 2 * TILEB) + (w * 64 + lane) * (NTE * 4 + 2);
    if (kg == 1) {
      xm[0] = m_q[0];
      xm[1] = l_q[0];
#pragma unroll
      for (int t = 0; t < NTE; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) xm[2 + 4 * t + i] = o[0][t][i];
    }
    __syncthreads();
    if (kg == 0) {
      const float m1 = xm[0], l1 = xm[1];
      const float mn = fmaxf(m_q[0], m1);
      const float s0 = m_q[0] == -INFINITY ? 0.f : __expf(m_q[0] - mn), s1 = m1 == -INFINITY ? 0.f : __expf(m1 - mn);
      l_q[0] = l_q[0] * s0 + l1 * s1;
      m_q[0] = mn;
#pragma unroll
      for (int t = 0; t < NTE; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) o[0][t][i] = o[0][t][i] * s0 + xm[2 + 4 * t + i] * s1;
    }
  }
#ifdef ATTN_STAMPS
  {
    volatile float sink = o[0][0][0];  // the P.V MFMAs retired
    (void)sink;
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
      st_lds[16 * 8 + 1] = __builtin_amdgcn_s_memtime();
      st_lds[16 * 8 + 2] = (unsigned long long)ntile;
      for (int i = 0; i < 17 * 8; i++) g_attn_stamps[blockIdx.x * 17 * 8 + i] = st_lds[i];
    }
  }
#endif
  if (QG == 1 && nspl > 1) {
    // split partial (running max, sum, unnormalised context) of the block's 64 queries, write-through:
    // record [m, l, -, -, o[0..hd)] per (split, query); the block drawing the last ticket of its (row,
    // head, query tile) merges the splits in split order
    const int rs = hd + 4;
    const int nqt = (a.S + QB - 1) / QB;
    const size_t item = ((size_t)pair * nqt + qt);
    const __amdgpu_buffer_rsrc_t rp = pf_rsrc(a.pf_ws + item * nspl * QB * rs);
    const int ql = w * 16 + r;
    const uint32_t rec = (uint32_t)((spl * QB + ql) * rs) * 4;
    if (kg == 0) {
      if (g == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m_q[0]), rp, rec, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l_q[0]), rp, rec + 4, 0, 16);
      }
#pragma unroll
      for (int t = 0; t < NTE; t++) {
        const int d = t * 16 + 4 * g;
        if (d < hd) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, o[0][t]), rp, rec + (4 + d) * 4, 0, 16);
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
    if (tid >= 256) return;  // the merge takes 4 threads per query
    const int qm = tid >> 2, j = tid & 3, nc = hd / 4;
    constexpr int G = 4, NC = 8;  // chunks per thread: ceil(128 / 4 / 4)
    float M = -INFINITY, Lsum = 0.f;
    f32x4 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < nspl; s0 += G) {
      float mg[G], lg[G];
      f32x4 og[G][NC];
#pragma unroll
      for (int uu = 0; uu < G; uu++) {
        const uint32_t rc = (uint32_t)((min(s0 + uu, nspl - 1) * QB + qm) * rs) * 4;
        mg[uu] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, rc, 0, 16));
        lg[uu] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, rc + 4, 0, 16));
#pragma unroll
        for (int c = 0; c < NC; c++)
          og[uu][c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rp, rc + (4 + 4 * min(j + 4 * c, nc - 1)) * 4, 0, 16));
      }
      float mn = M;
#pragma unroll
      for (int uu = 0; uu < G; uu++)
        if (s0 + uu < nspl) mn = fmaxf(mn, mg[uu]);
      const float sc = M == -INFINITY ? 0.f : __expf(M - mn);  // mn is finite: split 0 holds key 0
      Lsum *= sc;
#pragma unroll
      for (int c = 0; c < NC; c++) acc[c] *= sc;
#pragma unroll
      for (int uu = 0; uu < G; uu++) {
        // a split past the query's keys (m = -inf) or past nspl weighs 0
        const float wu = (s0 + uu < nspl && mg[uu] != -INFINITY) ? __expf(mg[uu] - mn) : 0.f;
        Lsum += wu * lg[uu];
#pragma unroll
        for (int c = 0; c < NC; c++) acc[c] += wu * og[uu][c];
      }
      M = mn;
    }
    const int q = qt * QB + qm;
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
  // context rows through LDS (the wave's own 16 x 128 bf16 region in group 0's stage 0), then 16-B row stores
  if (kg != 0) return;
  if constexpr (KG == 1) __syncthreads();  // (KG = 2: the merge's barriers already retired every ring read)
  bf16* cs = reinterpret_cast<bf16*>(smem) + w * 16 * QG * 128;
#pragma unroll
  for (int j = 0; j < QG; j++) {
    const float inv = 1.0f / l_q[j];
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int t = 0; t < NTE; t++) {
      bf16x4 v4;
#pragma unroll
      for (int i = 0; i < 4; i++) v4[i] = (bf16)(o[j][t][i] * inv);
      *reinterpret_cast<bf16x4*>(cs + (16 * j + r) * 128 + t * 16 + 4 * g) = v4;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes before its reads
#pragma unroll
  for (int i = 0; i < 4 * QG; i++) {
    const int c = i * 64 + lane, ql = c >> 4, ch = c & 15, q = q0 + ql;
    if (ch < nch && q < a.S)
      *reinterpret_cast<bf16x8*>((bf16*)a.ctx_out + ((size_t)b * a.S + q) * a.hidden + head * hd + ch * 8) =
          *reinterpret_cast<const bf16x8*>(cs + ql * 128 + ch * 8);
  }
}

// Split-KV when the grid would leave CU slots idle: the unit count is nqt x pairs x nspl with nspl = ceil(key tiles
// / pf_tiles), taken when nqt x pairs < max_units (the blocks co-resident: 2 per CU at 64 KB of LDS); NSTG LDS stages.
void attn_prefill_tr_launch(const AttnArgs& a, hipStream_t s, int nstg, int pf_tiles, int max_units, int kgroups,
                            int qgroups) {
  const int P = a.B * a.n_head;
  // qgroups < 0: two query groups per wave (128-query blocks, half the LDS reads per MFMA) when that grid still has
  // >= 512 blocks (two per CU) of full query groups; no key split, one key group.  tools/attn_prefill_bench.hip
  // (profiles/r05_attn_prefill_qg.txt): bloom-7b1 16 rows x 1024 tokens after 1024 cached 1326 -> 840 us, 4 rows x
  // 1024 tokens 95.8 -> 74.3 us; at 256 blocks (7b1 2 rows x 512) one group is faster (20.8 vs 23.1 us)
  if (qgroups < 0) qgroups = (a.S >= 128 && (long)((a.S + 127) / 128) * P >= 512) ? 2 : 1;
  if (qgroups == 2) {
    const int U2 = (a.S + 127) / 128;
    const dim3 g2(P * U2);
    const int xg2 = P % 8 == 0 ? 1 : 0;
    auto go2 = [&](auto hc) {
      constexpr int HDE = decltype(hc)::value;
      attn_prefill_tr_kernel<2, HDE, 1, 2><<<g2, 256, 0, s>>>(a, 1, U2, xg2);
    };
    if (a.head_dim <= 64) go2(IntC<64>{});
    else if (a.head_dim <= 96) go2(IntC<96>{});
    else go2(IntC<128>{});
    return;
  }
  constexpr int QB = 64;
  const int nqt = (a.S + QB - 1) / QB;
  const int ktiles = (a.pf_past_max + a.S + 63) / 64;  // the last query tile's, longest row
  const int pt = pf_tiles < 0 ? a.pf_tiles : pf_tiles;
  int nspl = 1;
  if (pt > 0 && a.pf_ws && a.pf_tickets && (long)nqt * P < max_units && ktiles > pt) {
    nspl = (ktiles + pt - 1) / pt;
    const size_t need = (size_t)P * nqt * nspl * QB * (a.head_dim + 4);
    if (need > a.pf_cap || (long)P * nqt > a.pf_ntickets) nspl = 1;
  }
  // kgroups < 0: two key groups per block (8 waves; each group walks alternate key tiles of the query tile, the
  // groups merge at the end) when the grid is one unsplit block per CU or fewer and the long query tiles see >= 8
  // key tiles -- bloom-7b1 / 3b at one row x 512 tokens 16.95 -> 15.8 / 14.7 -> 13.8 us; shorter contexts and
  // fuller grids are faster with one group (profiles/r05_attn_prefill_ab.txt)
  if (kgroups < 0) kgroups = (nspl == 1 && (long)nqt * P <= 256 && ktiles >= 8) ? 2 : 1;
  AttnArgs b = a;
  b.pf_tiles = pt;
  const int U = nqt * nspl;
  const dim3 g(P * U);
  const int xg = P % 8 == 0 ? 1 : 0;
  auto go = [&](auto hc) {
    constexpr int HDE = decltype(hc)::value;
    if (kgroups == 2) attn_prefill_tr_kernel<2, HDE, 2><<<g, 512, 0, s>>>(b, nspl, U, xg);
    else if (nstg == 3) attn_prefill_tr_kernel<3, HDE, 1><<<g, 256, 0, s>>>(b, nspl, U, xg);
    else attn_prefill_tr_kernel<2, HDE, 1><<<g, 256, 0, s>>>(b, nspl, U, xg);
  };
  if (a.head_dim <= 64) go(IntC<64>{});
  else if (a.head_dim <= 96) go(IntC<96>{});
  else go(IntC<128>{});
}

