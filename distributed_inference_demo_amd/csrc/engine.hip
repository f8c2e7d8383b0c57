// engine.hip — the persistent decode engine: every decoder block of a stage for one decode step
// (S = 1, batch M <= 2, bf16) in ONE launch on gfx950.
//
// Why: at batch 1 a layer is five dependent weight-streaming launches, and each pays
// a kernel boundary, a first-byte latency and a drain tail on ~1-3 us of actual streaming.  The
// weights do not depend on the activations, so here one workgroup per CU (256 x 1024 threads, all
// resident) streams its share of every layer through a register ring that runs ahead across the
// phase boundaries, and each phase only waits for its activations.
//
// Roles inside a workgroup (one per CU, block b):
//   waves 4..15 ("compute"): own the weight units of block b (1 KB = 64 lanes x 16 B of one weight
//     row, non-temporal loads), R in flight per wave (Ring): dot the phase's units against the
//     activations in LDS, one float per (unit, row) to LDS.  They issue no other global load, so the
//     in-order vmcnt never makes them wait for anything but the weights they are about to use.
//   wave 0 ("I/O"): waits for the phase's input vector and stages it in LDS (LayerNorm on the way).
//   wave 1 ("publisher"): after the compute waves are done sums the unit results, runs the epilogue
//     (bias, residual, GELU, q/K/V routing, attention merges) and publishes its rows.  Loads and stores
//     live on different waves: with a write-through store pending the compiler waits vmcnt(0) before
//     using any load, so one wave doing both put every sweep behind the previous phase's stores.
//   waves 2..3 ("attention"): decode attention of this block's (head, 64-position split); the
//     cached rows are requested at the start of the layer, before the QKV edge.
//
// Per layer l (modeling_bloom.py BloomBlock; the arithmetic and bf16 storage points of the launch path
// in kernels.hip):
//   A  x -> LN_in -> QKV rows of b (+ bias) -> q, K/V cache; q/k/v granules          edge QKV(l)
//   B  attention blocks (head, split): q.k / ALiBi / fp32 softmax partial -> granules; block
//      (head, split 0) merges the head's splits -> ctx[head] granules                 edges PART, CTX
//   C  ctx -> dense rows of b, + bias + x -> x1 granules                             edge X1(l)
//   D  x1 -> LN_post -> fc1 rows of b, + bias, GELU -> g granules                    edge G(l)
//   E  g -> fc2 rows of b, + bias + x1 -> x2 granules (the next layer's x); the last layer writes
//      the stage output
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", R2 "the data IS the flag"; gfx950 / ROCm 7.2): every
// handed-off value travels as an 8-byte granule {value, tag} written by ONE sc1 store; the consumer
// re-reads the granules (16-B sc1 loads, two granules each, never nt) until every tag equals the
// edge's epoch, and then holds the values -- no counter, no drain, no second load.  The epoch of edge
// e of layer l is 0x80000000 | ((gen * L + l) * 8 + e): `gen` is a launch counter the block that
// finishes last advances, so no granule buffer ever needs clearing (they start zeroed, a tag that
// never matches).  Every spin is bounded (200 ms): on expiry the block records it in `status` and
// stops waiting, so the grid always drains.
#include <type_traits>
#include "common.h"
#include "kernels.h"

namespace {

constexpr int kG = 256;                      // workgroups: one per CU
constexpr int kWaves = 16, kIO = 4, kCW = kWaves - kIO;
constexpr int kThreads = kWaves * 64;
// attention: waves kAttn0.. (kNAttn of them); a block takes PB = 64 / MM cached positions of one head
// (kNAttn waves x 4 rows x T loads); at most kMaxSplit splits per head (contexts <= 1024 at one row,
// <= 512 at two)
constexpr int kAttn0 = 2, kNAttn = 2;
template <int MM> struct AttnGeom { static constexpr int PB = 64 / MM, T = PB / (4 * kNAttn); };
constexpr int kMaxSplit = 16;
constexpr int kRec = 130;                    // granules per split record: max, sum, acc[<= 128]
enum Edge { E_X2 = 0, E_QKV = 1, E_PART = 2, E_CTX = 3, E_X1 = 4, E_G = 5 };
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms of s_memrealtime (100 MHz)

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
// 16-B sc1 load (L1 bypass): two granules another workgroup published in this launch
__device__ __forceinline__ u32x4v ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ uint32_t ld4_sc1(const void* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4_sc1(void* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one granule {value, tag}: ONE aligned 8-byte sc1 store
__device__ __forceinline__ void put_granule(void* p, uint32_t tag, uint32_t value) {
  __hip_atomic_store((gu64*)p, ((unsigned long long)tag << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Workgroup barrier that waits for LDS only: a compute wave's outstanding weight loads must not be
// drained here, which __syncthreads()' release fence would do.
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// An opaque copy of a uniform pointer: what is derived from it is computed where it is used, not hoisted
// out of the layer loop and held (in SGPRs, then spilled) across every phase.
template <typename T> __device__ __forceinline__ T* fresh(T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16 x = (bf16)a, y = (bf16)b;
  return (uint32_t)__builtin_bit_cast(unsigned short, x) | ((uint32_t)__builtin_bit_cast(unsigned short, y) << 16);
}
__device__ __forceinline__ float bf16_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t v) { return __uint_as_float(v & 0xFFFF0000u); }
__device__ __forceinline__ float bf16_at(const void* p, int i) {
  return __uint_as_float((uint32_t)((const unsigned short*)p)[i] << 16);
}

// Layer tensors: one arena, every tensor 256-B aligned in canonical order (stage.hip init_stage); for
// h % 128 == 0 every size is a multiple of 256 B, so the offsets inside a layer are constants of H.
template <int H> struct LayerOff {
  static constexpr size_t LN1_G = 0, LN1_B = LN1_G + 2 * H, QKV_W = LN1_B + 2 * H, QKV_B = QKV_W + 6ull * H * H,
                          DENSE_W = QKV_B + 6 * H, DENSE_B = DENSE_W + 2ull * H * H, LN2_G = DENSE_B + 2 * H,
                          LN2_B = LN2_G + 2 * H, FC1_W = LN2_B + 2 * H, FC1_B = FC1_W + 8ull * H * H,
                          FC2_W = FC1_B + 8 * H, FC2_B = FC2_W + 8ull * H * H, END = FC2_B + 2 * H;
};
// Workspace (EngineArgs::ws, zeroed at init): control words, then granule buffers sized for 2 rows.
//   x2, x1: one fp32 granule per element; q, k, v (the new position), ctx: one bf16 pair per granule;
//   g: bf16 pairs; part: [n_head][kMaxSplit][2][kRec] fp32 split records.
struct Ctl { static constexpr int GEN = 0, DONE = 16, STATUS = 32, STATUS_LAST = 33; };
template <int H> struct WsOff {
  static constexpr size_t GX2 = 256, GX1 = GX2 + 16 * H, GQ = GX1 + 16 * H, GK = GQ + 8 * H, GV = GK + 8 * H,
                          GCTX = GV + 8 * H, GG = GCTX + 8 * H, GPART = GG + 32 * H;
};

__device__ __forceinline__ uint32_t tag_of(uint32_t gen, int L, int l, int e) {
  return 0x80000000u | (((gen * (uint32_t)L + (uint32_t)l) * 8u + (uint32_t)e) & 0x7FFFFFFFu);
}

// Wave-uniform bounded sweep: pairs p = c * 64 + lane (c < NC, p < npairs) of two granules each, at byte
// offset off(p) in r, re-read until every tag equals `tag`; then v[c] = (value0, value1).  `dead` (LDS)
// short-circuits every later sweep of the block once one expired.
template <int NC, typename OFF>
__device__ bool sweep(__amdgpu_buffer_rsrc_t r, int npairs, OFF off, uint32_t tag, uint32_t (&v)[NC][2],
                      unsigned* status, int* dead) {
  const int lane = threadIdx.x & 63;
  if (*(volatile int*)dead) return false;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const int p = c * 64 + lane;
      if (p < npairs) {
        const u32x4v x = ld16_sc1(r, off(p));
        v[c][0] = x.x;
        v[c][1] = x.z;
        ok = ok && x.y == tag && x.w == tag;
      }
    }
    if (__all(ok)) return true;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
      if (lane == 0) { st4_sc1(status, 1u); *(volatile int*)dead = 1; }
      return false;
    }
  }
}

template <int H> struct Shape {
  static constexpr int KC1 = H / 512, KC2 = 4 * H / 512;               // 512-column chunks per row
  static constexpr int RQ = 3 * H / kG, RD = H / kG, R1 = 4 * H / kG, R2 = H / kG;  // rows per block
  static constexpr int UQ = RQ * KC1, UD = RD * KC1, U1 = R1 * KC1, U2 = R2 * KC2;  // units per block
  static constexpr int NQ = (UQ + kCW - 1) / kCW, ND = (UD + kCW - 1) / kCW;        // units per wave
  static constexpr int N1 = (U1 + kCW - 1) / kCW, N2 = (U2 + kCW - 1) / kCW;
  static constexpr int UMAX = UQ > U1 ? (UQ > U2 ? UQ : U2) : (U1 > U2 ? U1 : U2);
  static constexpr int NP = H / 128;                                    // fp32 granule pairs per lane per row
};

// LDS of one workgroup
template <int MM, int H> struct Smem {
  bf16 xs[MM * 4 * H];                   // the phase's activations (bf16): xn, ctx or g rows
  float xf[MM * H];                      // the residual rows (fp32): x during A..C, x1 during D..E
  float res[Shape<H>::UMAX * MM];        // one dot per (unit, row)
  bf16 qkv[MM][3][128];                  // attention: q, k and v of the new position (this head)
  float ap[kNAttn][MM][kRec];            // attention: per-wave (max, sum, acc[hd]) partials
  float wt[kMaxSplit];                   // attention: split weights of the merge
  float mg[kMaxSplit * MM * kRec];       // attention: the head's split records (merger block)
  int dead;
#ifdef BS_ENGINE_STAMPS
  unsigned long long stamps[64 * 5 * 6];
#endif
};

// ---- wave 0: a row's values in registers, NP pairs per lane (elements (c * 64 + lane) * 2 + {0, 1})
template <int NP>
__device__ __forceinline__ void ln_pairs(float (&v)[NP][2], float eps, int H) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NP; c++) s += v[c][0] + v[c][1];
  const float mean = wave_sum(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NP; c++) {
    const float d0 = v[c][0] - mean, d1 = v[c][1] - mean;
    q += d0 * d0 + d1 * d1;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int c = 0; c < NP; c++) { v[c][0] = (v[c][0] - mean) * rstd; v[c][1] = (v[c][1] - mean) * rstd; }
}
// y = ((x - mean) * rstd) * gamma + beta (nn.LayerNorm order), gamma/beta one bf16 pair
__device__ __forceinline__ float2 affine2(float a, float b, uint32_t g, uint32_t be) {
  return make_float2(a * bf16_lo(g) + bf16_lo(be), b * bf16_hi(g) + bf16_hi(be));
}

}  // namespace

typedef const __attribute__((address_space(4))) EngineArgs KArgs;  // kernarg segment: scalar loads

// Diagnostic builds only (tools/engine_timeline.hip defines BS_ENGINE_STAMPS): waves 0 and 1 of every
// block record s_memrealtime (100 MHz) at five points of every phase of every layer, in LDS (a global
// store would put a store in front of the I/O wave's loads); wave 0 copies them out at the end.
#ifdef BS_ENGINE_STAMPS
__device__ unsigned long long g_eng_stamps[256 * 64 * 5 * 6];
#define ESTAMP(l, ph, k)                                                                              \
  do {                                                                                              \
    if ((threadIdx.x & 63) == 0) sm->stamps[((l) * 5 + (ph)) * 6 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ESTAMP(l, ph, k) do {} while (0)
#endif

// The kernel argument, re-read from the kernarg segment where used (scalar loads, uniform), and the
// workgroup's LDS (dynamic, sizeof(Smem<MM, H>)).  A callee cannot name the kernarg segment itself (the
// intrinsic lowers to 0 outside the kernel), so the kernel passes its address and the callee rebuilds
// it wave-uniform.
__device__ __forceinline__ KArgs* kargs(uint64_t bits) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bits), hi = __builtin_amdgcn_readfirstlane((uint32_t)(bits >> 32));
  return (KArgs*)(((uint64_t)hi << 32) | lo);
}
extern __shared__ __attribute__((aligned(16))) char engine_lds[];
template <int MM, int H> __device__ __forceinline__ Smem<MM, H>* smem() { return (Smem<MM, H>*)engine_lds; }

// What every wave derives at kernel start: the rows' positions, this block's attention task, the epoch.
template <int MM> struct Step {
  int past[MM];
  int nsplit, ahead, asplit;
  bool attn;
  uint32_t gen;
};
template <int MM>
__device__ __forceinline__ Step<MM> step_of(KArgs* a, int b) {
  Step<MM> st;
  int pmax = 0;
#pragma unroll
  for (int m = 0; m < MM; m++) { st.past[m] = a->past_dev[m]; pmax = max(pmax, st.past[m]); }
  st.nsplit = (pmax + 1 + AttnGeom<MM>::PB - 1) / AttnGeom<MM>::PB;
  st.attn = b < a->n_head * st.nsplit;
  st.ahead = st.attn ? b / st.nsplit : 0;
  st.asplit = st.attn ? b % st.nsplit : 0;
  st.gen = __builtin_amdgcn_readfirstlane(((const unsigned*)a->ws)[Ctl::GEN]);  // set by the previous launch
  return st;
}

// ============ compute waves (4..15): the weight stream through a register ring
// A wave's units of one layer, in use order: NQ QKV, ND dense, N1 fc1, N2 fc2 (padded to a multiple of
// the ring depth R).  The ring keeps R units in flight: consuming unit j re-issues its registers for unit
// j + R -- of this layer, or of the next one across the layer boundary -- so every phase starts with its
// first units landed or in flight while the edge before it is being waited for ("prefetch credit"), and
// the CU never has more than kCW * R KB of weight requests queued (a whole layer ahead -- 221 KB per CU
// at bloom-1b1 -- stalled the issuing waves and the I/O wave's own loads behind the queue).
template <int H> struct Ring {
  using S = Shape<H>;
  static constexpr int R = 4;
  static constexpr int NU = S::NQ + S::ND + S::N1 + S::N2;
  static constexpr int NUP = (NU + R - 1) / R * R;
  static constexpr int B1 = S::NQ, B2 = S::NQ + S::ND, B3 = S::NQ + S::ND + S::N1;  // phase starts
};

template <int MM, int H>
__device__ __attribute__((noinline)) void role_compute(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<MM, H>* sm = smem<MM, H>();
  const bool attn = step_of<MM>(a, blockIdx.x).attn;
  using S = Shape<H>;
  using LO = LayerOff<H>;
  using RG = Ring<H>;
  constexpr int R = RG::R;
  const int lane = threadIdx.x & 63, cw = (threadIdx.x >> 6) - kIO, b = blockIdx.x;
  const int L = a->L;
  const size_t ls = a->layer_stride;
  const char* wl = a->wl;
  const bf16* blk[4] = {(const bf16*)(wl + LO::QKV_W) + (size_t)b * S::RQ * H,
                        (const bf16*)(wl + LO::DENSE_W) + (size_t)b * S::RD * H,
                        (const bf16*)(wl + LO::FC1_W) + (size_t)b * S::R1 * H,
                        (const bf16*)(wl + LO::FC2_W) + (size_t)b * S::R2 * 4 * H};
  // unit j of the layer -> (phase, wave-local index); pads re-read the layer's last unit
  auto ph_of = [](int j) { return j < RG::B1 ? 0 : j < RG::B2 ? 1 : j < RG::B3 ? 2 : 3; };
  auto idx_of = [](int j) {
    const int jj = j < RG::NU ? j : RG::NU - 1;
    return jj < RG::B1 ? jj : jj < RG::B2 ? jj - RG::B1 : jj < RG::B3 ? jj - RG::B2 : jj - RG::B3;
  };
  auto umax = [](int ph) { return ph == 0 ? S::UQ : ph == 1 ? S::UD : ph == 2 ? S::U1 : S::U2; };
  auto addr = [&](int j, size_t off) {
    const int jj = j < RG::NU ? j : RG::NU - 1;
    const int ph = ph_of(jj), u = min(cw + kCW * idx_of(jj), umax(ph) - 1);
    return (const bf16*)((const char*)blk[ph] + off) + (size_t)u * 512 + lane * 8;
  };
  bf16x8 w[R];
#pragma unroll
  for (int j = 0; j < R; j++) w[j] = wload<1>(addr(j, 0));
  for (int l = 0; l < L; l++) {
    const size_t cur = (size_t)l * ls, nxt = (size_t)min(l + 1, L - 1) * ls;  // last layer: harmless re-reads
#pragma unroll
    for (int j = 0; j < RG::NUP; j++) {
      if (j == 0) bar();                                              // A: S2
      if (j == RG::B1) { bar(); if (attn) { bar(); bar(); bar(); } bar(); }  // A: S3; B: S1'-S3'; C: S2
      if (j == RG::B2) { bar(); bar(); }                              // C: S3; D: S2
      if (j == RG::B3) { bar(); bar(); }                              // D: S3; E: S2
      if (j < RG::NU) {
        const int ph = ph_of(j), u = cw + kCW * idx_of(j);
        if (u < umax(ph)) {
          const int K = ph == 3 ? 4 * H : H, KC = ph == 3 ? S::KC2 : S::KC1;
          const int c = u % KC;
#pragma unroll
          for (int m = 0; m < MM; m++) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(sm->xs + m * K + c * 512 + lane * 8);
            const float v = wave_sum(dot8(w[j % R], x, 0.f));
            if (lane == 0) sm->res[u * MM + m] = v;
          }
        }
      }
      const int jn = j + R;
      w[j % R] = wload<1>(jn < RG::NUP ? addr(jn, cur) : addr(jn - RG::NUP, nxt));
    }
    bar();  // E: S3
  }
}

// ============ attention waves (2..3): decode attention of one (head, split) per attention block
template <int MM, int H>
__device__ __attribute__((noinline)) void role_attn(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<MM, H>* sm = smem<MM, H>();
  const Step<MM> st = step_of<MM>(a, blockIdx.x);
  constexpr int PB = AttnGeom<MM>::PB, T = AttnGeom<MM>::T;
  const int lane = threadIdx.x & 63, kw = (threadIdx.x >> 6) - kAttn0;
  const int L = a->L, hd = a->hd, nh = a->n_head;
  const int grp = lane >> 4, dl = lane & 15;  // 16 lanes per cached row, 8 dims each; 4 rows per load
  const bool dval = dl * 8 < hd;
  const int doff = dval ? dl * 8 : 0;
  const float slope = st.attn ? a->slopes[st.ahead] : 0.f;
  auto pos = [&](int t) { return kw * 4 + grp + 4 * kNAttn * t; };  // split-local position of load t
  for (int l = 0; l < L; l++) {
    u32x4v kr[MM][T], vr[MM][T];
    KArgs* A = fresh(a);
    if (st.attn) {
      // the cached rows (positions < past) of this block's split: requested before the QKV edge
      const bf16* kl = (const bf16*)(A->kv + (size_t)l * A->kv_layer_stride);
      const bf16* vl = (const bf16*)((const char*)kl + A->kv_half);
      const int mctx = A->max_ctx;
      const size_t hb = ((size_t)A->slot * nh + st.ahead) * mctx;
#pragma unroll
      for (int m = 0; m < MM; m++) {
        const size_t rb = (hb + (size_t)m * nh * mctx) * hd;
#pragma unroll
        for (int t = 0; t < T; t++) {
          const int p = min(st.asplit * PB + pos(t), max(st.past[m] - 1, 0));
          kr[m][t] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(kl + rb + (size_t)p * hd + doff));
          vr[m][t] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(vl + rb + (size_t)p * hd + doff));
        }
      }
    }
    bar(); bar();  // A: S2, S3
    if (st.attn) {
      bar();  // B: S1' -- q, k, v of the new position in LDS
      const float inv_norm = A->inv_norm;
#pragma unroll
      for (int m = 0; m < MM; m++) {
#pragma unroll
        for (int t = 0; t < T; t++) {
          if (st.asplit * PB + pos(t) == st.past[m]) {
            kr[m][t] = *reinterpret_cast<const u32x4v*>(&sm->qkv[m][1][doff]);
            vr[m][t] = *reinterpret_cast<const u32x4v*>(&sm->qkv[m][2][doff]);
          }
        }
        const u32x4v qraw = *reinterpret_cast<const u32x4v*>(&sm->qkv[m][0][doff]);
        const float q8[8] = {bf16_lo(qraw.x), bf16_hi(qraw.x), bf16_lo(qraw.y), bf16_hi(qraw.y),
                             bf16_lo(qraw.z), bf16_hi(qraw.z), bf16_lo(qraw.w), bf16_hi(qraw.w)};
        float sc[T];
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < T; t++) {
          const u32x4v k = kr[m][t];
          float d = q8[0] * bf16_lo(k.x) + q8[1] * bf16_hi(k.x) + q8[2] * bf16_lo(k.y) + q8[3] * bf16_hi(k.y) +
                    q8[4] * bf16_lo(k.z) + q8[5] * bf16_hi(k.z) + q8[6] * bf16_lo(k.w) + q8[7] * bf16_hi(k.w);
          d = dval ? d : 0.f;
          d += dpp_f<0xB1>(d);   // sum over the row's 16 lanes: xor 1, xor 2, rotate 4, rotate 8
          d += dpp_f<0x4E>(d);
          d += dpp_f<0x124>(d);
          d += dpp_f<0x128>(d);
          const int j = pos(t);
          const int p = st.asplit * PB + j;
          const bool live = j < PB && p <= st.past[m];
          sc[t] = live ? slope * (float)p + inv_norm * d : -INFINITY;
          mx = fmaxf(mx, sc[t]);
        }
        mx = wave_max(mx);
        float e[T], lsum = 0.f;
#pragma unroll
        for (int t = 0; t < T; t++) {
          e[t] = sc[t] == -INFINITY ? 0.f : __expf(sc[t] - mx);
          lsum += e[t];
        }
        lsum = wave_sum(dl == 0 ? lsum : 0.f);
        float acc[8];
#pragma unroll
        for (int jj = 0; jj < 8; jj++) acc[jj] = 0.f;
#pragma unroll
        for (int t = 0; t < T; t++) {
          const u32x4v v = vr[m][t];
          acc[0] += e[t] * bf16_lo(v.x); acc[1] += e[t] * bf16_hi(v.x);
          acc[2] += e[t] * bf16_lo(v.y); acc[3] += e[t] * bf16_hi(v.y);
          acc[4] += e[t] * bf16_lo(v.z); acc[5] += e[t] * bf16_hi(v.z);
          acc[6] += e[t] * bf16_lo(v.w); acc[7] += e[t] * bf16_hi(v.w);
        }
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
          acc[jj] += __shfl_xor(acc[jj], 16, 64);
          acc[jj] += __shfl_xor(acc[jj], 32, 64);
        }
        if (grp == 0 && dval) {
#pragma unroll
          for (int jj = 0; jj < 8; jj++) sm->ap[kw][m][2 + dl * 8 + jj] = acc[jj];
        }
        if (lane == 0) { sm->ap[kw][m][0] = mx; sm->ap[kw][m][1] = lsum; }
      }
      bar(); bar();  // B: S2', S3'
    }
    bar(); bar();  // C
    bar(); bar();  // D
    bar(); bar();  // E
  }
}

// ============ wave 0: every load of handed-off values (granule sweeps) and their staging in LDS.  It
// issues no global store, so its loads never queue behind write-through stores (with stores pending
// the compiler waits vmcnt(0) before using any load).
template <int MM, int H>
__device__ __attribute__((noinline)) void role_io(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<MM, H>* sm = smem<MM, H>();
  const Step<MM> st = step_of<MM>(a, blockIdx.x);
  using S = Shape<H>;
  using LO = LayerOff<H>;
  using WO = WsOff<H>;
  constexpr int NP = S::NP;
  const int lane = threadIdx.x & 63;
  const int L = a->L, hd = a->hd;
  const size_t ls = a->layer_stride;
  unsigned* status = (unsigned*)(a->ws) + Ctl::STATUS;
  if (lane == 0) sm->dead = 0;
  // fp32 vector of granules (x2 / x1): row m's NP pairs per lane -> v
  auto sweep_row = [&](char* ws, size_t off, int m, uint32_t tag, float (&v)[NP][2]) {
    uint32_t raw[NP][2];
    sweep<NP>(rsrc(ws + off), H / 2, [&](int p) { return (uint32_t)((m * H / 2 + p) * 16); }, tag, raw, status, &sm->dead);
#pragma unroll
    for (int c = 0; c < NP; c++) { v[c][0] = __uint_as_float(raw[c][0]); v[c][1] = __uint_as_float(raw[c][1]); }
  };
  // bf16-pair vector of granules (ctx: n = H, g: n = 4H elements per row) -> xs[m * n ..]; a row in one
  // sweep (every load of a pass in flight together: a chunked sweep paid one round trip per chunk)
  auto sweep_bf16 = [&](char* ws, size_t off, int n, uint32_t tag) {
    constexpr int NC = H / 64;  // pairs per lane: a g row (4H elements = H pairs)
#pragma unroll 1
    for (int m = 0; m < MM; m++)
#pragma unroll 1
      for (int p0 = 0; p0 < n / 4; p0 += NC * 64) {
        uint32_t raw[NC][2];
        const int np = min(NC * 64, n / 4 - p0);
        sweep<NC>(rsrc(ws + off), np, [&](int p) { return (uint32_t)(((size_t)m * n / 2 + (p0 + p) * 2) * 8); }, tag, raw,
                  status, &sm->dead);
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const int p = c * 64 + lane;
          if (p < np) *reinterpret_cast<uint2*>(&sm->xs[m * n + (p0 + p) * 4]) = make_uint2(raw[c][0], raw[c][1]);
        }
      }
  };
  // gamma / beta of a LayerNorm, requested before the sweep it follows (a load issued after the sweep
  // is one more memory round trip on the critical path)
  auto load_gb = [&](const bf16* g, const bf16* be, uint32_t (&gb)[NP][2]) {
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      gb[c][0] = *reinterpret_cast<const uint32_t*>(g + k);
      gb[c][1] = *reinterpret_cast<const uint32_t*>(be + k);
    }
  };
  // x (fp32, registers) -> xf, LN(x) * gamma + beta -> xs (bf16)
  auto stage_ln = [&](int m, float (&v)[NP][2], const uint32_t (&gb)[NP][2], float eps) {
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      *reinterpret_cast<float2*>(&sm->xf[m * H + k]) = make_float2(v[c][0], v[c][1]);
    }
    ln_pairs<NP>(v, eps, H);
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      const float2 y = affine2(v[c][0], v[c][1], gb[c][0], gb[c][1]);
      *reinterpret_cast<uint32_t*>(&sm->xs[m * H + k]) = pack_bf16x2(y.x, y.y);
    }
  };

  for (int l = 0; l < L; l++) {
    // ---------------- A: x -> LN_in -> xs
    ESTAMP(l, 0, 0);
    {
      KArgs* A = fresh(a);
      const char* wl = A->wl + (size_t)l * ls;
      const float eps = A->eps;
      uint32_t gb[NP][2];
      load_gb((const bf16*)(wl + LO::LN1_G), (const bf16*)(wl + LO::LN1_B), gb);
#pragma unroll 1
      for (int m = 0; m < MM; m++) {
        float v[NP][2];
        if (l > 0) {
          sweep_row(A->ws, WO::GX2, m, tag_of(st.gen, L, l - 1, E_X2), v);
        } else if (A->x_in) {
#pragma unroll
          for (int c = 0; c < NP; c++) {
            const float2 t = *reinterpret_cast<const float2*>(A->x_in + m * H + (c * 64 + lane) * 2);
            v[c][0] = t.x; v[c][1] = t.y;
          }
        } else {
          // first stage: word_embeddings[id] -> word_embeddings_layernorm (fp32) is the residual stream
          const bf16* row = (const bf16*)A->wemb + (size_t)A->ids[m] * H;
#pragma unroll
          for (int c = 0; c < NP; c++) {
            const uint32_t r = *reinterpret_cast<const uint32_t*>(row + (c * 64 + lane) * 2);
            v[c][0] = bf16_lo(r); v[c][1] = bf16_hi(r);
          }
          ln_pairs<NP>(v, eps, H);
#pragma unroll
          for (int c = 0; c < NP; c++) {
            const int k = (c * 64 + lane) * 2;
            const float2 y = affine2(v[c][0], v[c][1], *reinterpret_cast<const uint32_t*>((const bf16*)A->emb_g + k),
                                     *reinterpret_cast<const uint32_t*>((const bf16*)A->emb_b + k));
            v[c][0] = y.x; v[c][1] = y.y;
          }
        }
        ESTAMP(l, 0, 1);
        stage_ln(m, v, gb, eps);
      }
    }
    bar();  // S2: xs ready
    ESTAMP(l, 0, 2);
    bar();  // S3
    // ---------------- B: the new position's q, k, v of this head -> LDS; the merger also stages the records
    if (st.attn) {
      ESTAMP(l, 1, 0);
      {
        KArgs* A = fresh(a);
        const int per = hd / 4, np = 3 * MM * per;  // granule pairs
        uint32_t raw[3][2];
        auto poff = [&](int p) {
          const int which = p / (MM * per), r = p - which * MM * per, m = r / per, q = r - m * per;
          return (uint32_t)((size_t)which * 8 * H + ((size_t)m * H / 2 + st.ahead * hd / 2 + q * 2) * 8);
        };
        sweep<3>(rsrc(A->ws + WO::GQ), np, poff, tag_of(st.gen, L, l, E_QKV), raw, status, &sm->dead);
#pragma unroll
        for (int c = 0; c < 3; c++) {
          const int p = c * 64 + lane;
          if (p < np) {
            const int which = p / (MM * per), r = p - which * MM * per, m = r / per, q = r - m * per;
            *reinterpret_cast<uint2*>(&sm->qkv[m][which][q * 4]) = make_uint2(raw[c][0], raw[c][1]);
          }
        }
      }
      ESTAMP(l, 1, 1);
      bar();  // S1'
      bar();  // S2': wave 1 publishes this split's record
      if (st.asplit == 0) {
        // the head's merger: every split's record (granule pairs) -> LDS mg
        KArgs* A = fresh(a);
        char* part = A->ws + WO::GPART + (size_t)st.ahead * kMaxSplit * MM * kRec * 8;
        const int rp2 = (hd + 2) / 2;             // pairs a record uses: (max, sum), acc[hd]
        const int npair = st.nsplit * MM * rp2;
        constexpr int NC = 11;
        const __amdgpu_buffer_rsrc_t rp = rsrc(part);
        const uint32_t tp = tag_of(st.gen, L, l, E_PART);
#pragma unroll 1
        for (int p0 = 0; p0 < npair; p0 += NC * 64) {
          uint32_t raw[NC][2];
          const int np = min(NC * 64, npair - p0);
          auto roff = [&](int p) {
            const int q = p0 + p, r = q / rp2;
            return (uint32_t)((r * kRec + (q - r * rp2) * 2) * 8);
          };
          sweep<NC>(rp, np, roff, tp, raw, status, &sm->dead);
#pragma unroll
          for (int c = 0; c < NC; c++) {
            const int p = c * 64 + lane;
            if (p < np) {
              const int q = p0 + p, r = q / rp2;
              *reinterpret_cast<float2*>(&sm->mg[r * kRec + (q - r * rp2) * 2]) =
                  make_float2(__uint_as_float(raw[c][0]), __uint_as_float(raw[c][1]));
            }
          }
        }
      }
      bar();  // S3': records staged (merger)
    }
    // ---------------- C: ctx -> xs
    ESTAMP(l, 2, 0);
    sweep_bf16(fresh(a)->ws, WO::GCTX, H, tag_of(st.gen, L, l, E_CTX));
    ESTAMP(l, 2, 1);
    bar();  // S2
    ESTAMP(l, 2, 2);
    bar();  // S3
    // ---------------- D: x1 -> xf, LN_post -> xs
    ESTAMP(l, 3, 0);
    {
      KArgs* A = fresh(a);
      const char* wl = A->wl + (size_t)l * ls;
      const float eps = A->eps;
      uint32_t gb[NP][2];
      load_gb((const bf16*)(wl + LO::LN2_G), (const bf16*)(wl + LO::LN2_B), gb);
#pragma unroll 1
      for (int m = 0; m < MM; m++) {
        float v[NP][2];
        sweep_row(A->ws, WO::GX1, m, tag_of(st.gen, L, l, E_X1), v);
        ESTAMP(l, 3, 1);
        stage_ln(m, v, gb, eps);
      }
    }
    bar();  // S2
    ESTAMP(l, 3, 2);
    bar();  // S3
    // ---------------- E: g -> xs
    ESTAMP(l, 4, 0);
    sweep_bf16(fresh(a)->ws, WO::GG, 4 * H, tag_of(st.gen, L, l, E_G));
    ESTAMP(l, 4, 1);
    bar();  // S2
    ESTAMP(l, 4, 2);
    bar();  // S3
  }
#ifdef BS_ENGINE_STAMPS
  for (int i = lane; i < 64 * 5 * 6; i += 64) {  // wave 0's stamps (wave 1 copies its own)
    const int k = i % 6, ph = (i / 6) % 5;
    if (ph == 1 ? k < 2 : k < 4) g_eng_stamps[(size_t)blockIdx.x * 64 * 5 * 6 + i] = sm->stamps[i];
  }
#endif
}

// ============ wave 1: every epilogue and every global store (granules, K/V cache rows, the stage
// output).  The biases of a layer are loaded at the layer's start, ahead of its stores, so no load of
// this wave waits for a write-through store.
template <int MM, int H>
__device__ __attribute__((noinline)) void role_pub(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<MM, H>* sm = smem<MM, H>();
  const Step<MM> st = step_of<MM>(a, blockIdx.x);
  using S = Shape<H>;
  using LO = LayerOff<H>;
  using WO = WsOff<H>;
  const int lane = threadIdx.x & 63, b = blockIdx.x;
  const int L = a->L, hd = a->hd, nh = a->n_head;
  const size_t ls = a->layer_stride;
  // this lane's rows of each epilogue (lanes past a phase's rows read row 0 and never store)
  const int nq = b * S::RQ + 2 * min(lane, S::RQ / 2 - 1), nd = b * S::RD + min(lane, S::RD - 1);
  const int n1 = b * S::R1 + 2 * min(lane, S::R1 / 2 - 1), n2 = b * S::R2 + min(lane, S::R2 - 1);
  const int three = 3 * hd, qhead = nq / three, qrr = nq - qhead * three, qwhich = qrr / hd, qd = qrr - qwhich * hd;
  for (int l = 0; l < L; l++) {
    uint32_t bq, bd, b1, b2;  // raw bf16 bias (pairs for QKV and fc1)
    {
      KArgs* A = fresh(a);
      const char* wl = A->wl + (size_t)l * ls;
      bq = *reinterpret_cast<const uint32_t*>((const bf16*)(wl + LO::QKV_B) + nq);
      bd = ((const unsigned short*)(wl + LO::DENSE_B))[nd];
      b1 = *reinterpret_cast<const uint32_t*>((const bf16*)(wl + LO::FC1_B) + n1);
      b2 = ((const unsigned short*)(wl + LO::FC2_B))[n2];
    }
    bar(); bar();  // A: S2, S3
    {
      // QKV: lane j < RQ / 2 takes rows (2j, 2j + 1) of the block (never across a q/k/v segment): q, k, v
      // as granules for this step's attention; k, v also to the cache for the steps after
      KArgs* A = fresh(a);
      char* kl = (char*)A->kv + (size_t)l * A->kv_layer_stride;
      char* vl = kl + A->kv_half;
      char* gq = A->ws + WO::GQ;
      const int slot = A->slot, mctx = A->max_ctx;
      const uint32_t tag = tag_of(st.gen, L, l, E_QKV);
      if (lane < S::RQ / 2) {
#pragma unroll
        for (int m = 0; m < MM; m++) {
          float v0 = 0.f, v1 = 0.f;
#pragma unroll
          for (int c = 0; c < S::KC1; c++) {
            v0 += sm->res[((2 * lane) * S::KC1 + c) * MM + m];
            v1 += sm->res[((2 * lane + 1) * S::KC1 + c) * MM + m];
          }
          const uint32_t pk = pack_bf16x2(v0 + bf16_lo(bq), v1 + bf16_hi(bq));
          if (qwhich) {
            char* c = (qwhich == 1 ? kl : vl) + ((((size_t)(slot + m) * nh + qhead) * mctx + st.past[m]) * hd + qd) * 2;
            *reinterpret_cast<uint32_t*>(c) = pk;  // read by later launches only
          }
          put_granule(gq + (size_t)qwhich * 8 * H + ((size_t)m * H / 2 + (qhead * hd + qd) / 2) * 8, tag, pk);
        }
      }
    }
    ESTAMP(l, 0, 4);
    // ---------------- B
    if (st.attn) {
      bar(); bar();  // S1', S2': the attention waves' partials in LDS
      ESTAMP(l, 1, 2);
      KArgs* A = fresh(a);
      // merge the wave partials -> this split's record (max, sum, acc[hd]) as granules; lane: dims 2 * lane, + 1
      char* part = A->ws + WO::GPART + (size_t)st.ahead * kMaxSplit * MM * kRec * 8;
      const uint32_t tp = tag_of(st.gen, L, l, E_PART);
      const int d0 = 2 * lane;
      const bool dv = d0 < hd;
#pragma unroll 1
      for (int m = 0; m < MM; m++) {
        float M = -INFINITY;
#pragma unroll
        for (int k = 0; k < kNAttn; k++) M = fmaxf(M, sm->ap[k][m][0]);
        float Ls = 0.f, o0 = 0.f, o1 = 0.f;
        if (M != -INFINITY) {
#pragma unroll
          for (int k = 0; k < kNAttn; k++) {
            const float wgt = __expf(sm->ap[k][m][0] - M);
            Ls += wgt * sm->ap[k][m][1];
            if (dv) { o0 += wgt * sm->ap[k][m][2 + d0]; o1 += wgt * sm->ap[k][m][3 + d0]; }
          }
        }
        char* rec = part + ((size_t)st.asplit * MM + m) * kRec * 8;
        // every granule of the record is written (pads too), so the merger can wait for whole pairs
        put_granule(rec + (2 + d0) * 8, tp, __float_as_uint(dv ? o0 : 0.f));
        put_granule(rec + (3 + d0) * 8, tp, __float_as_uint(dv ? o1 : 0.f));
        if (lane == 0) {
          put_granule(rec, tp, __float_as_uint(M));
          put_granule(rec + 8, tp, __float_as_uint(Ls));
        }
      }
      ESTAMP(l, 1, 3);
      bar();  // S3': the merger's records staged in LDS by wave 0
      if (st.asplit == 0) {
        char* gctx = A->ws + WO::GCTX;
        const uint32_t tc = tag_of(st.gen, L, l, E_CTX);
#pragma unroll 1
        for (int m = 0; m < MM; m++) {
          const int t = min(lane, st.nsplit - 1);
          const float mt = sm->mg[(t * MM + m) * kRec], lt = sm->mg[(t * MM + m) * kRec + 1];
          const bool ok = lane < st.nsplit && mt != -INFINITY;
          const float M = wave_max(ok ? mt : -INFINITY);
          const float wgt = ok ? __expf(mt - M) : 0.f;
          const float Ls = wave_sum(wgt * (ok ? lt : 0.f));
          if (lane < kMaxSplit) sm->wt[lane] = wgt;
          if (dv) {
            float o0 = 0.f, o1 = 0.f;
            for (int u = 0; u < st.nsplit; u++) {
              const float wu = sm->wt[u];
              const float2 av = *reinterpret_cast<const float2*>(&sm->mg[(u * MM + m) * kRec + 2 + d0]);
              o0 += wu * av.x;
              o1 += wu * av.y;
            }
            put_granule(gctx + ((size_t)m * H / 2 + (st.ahead * hd + d0) / 2) * 8, tc, pack_bf16x2(o0 / Ls, o1 / Ls));
          }
        }
        ESTAMP(l, 1, 4);
      }
    }
    // ---------------- C: dense -> x1 = x + dense(ctx) + bias
    bar(); bar();  // S2, S3
    {
      KArgs* A = fresh(a);
      char* gx1 = A->ws + WO::GX1;
      const uint32_t tag = tag_of(st.gen, L, l, E_X1);
      if (lane < S::RD) {
#pragma unroll
        for (int m = 0; m < MM; m++) {
          float v = 0.f;
#pragma unroll
          for (int c = 0; c < S::KC1; c++) v += sm->res[(lane * S::KC1 + c) * MM + m];
          put_granule(gx1 + ((size_t)m * H + nd) * 8, tag, __float_as_uint((v + bf16_lo(bd)) + sm->xf[m * H + nd]));
        }
      }
    }
    ESTAMP(l, 2, 4);
    // ---------------- D: fc1 + GELU -> g
    bar(); bar();  // S2, S3
    {
      KArgs* A = fresh(a);
      char* gg = A->ws + WO::GG;
      const uint32_t tag = tag_of(st.gen, L, l, E_G);
      if (lane < S::R1 / 2) {
#pragma unroll
        for (int m = 0; m < MM; m++) {
          float v0 = 0.f, v1 = 0.f;
#pragma unroll
          for (int c = 0; c < S::KC1; c++) {
            v0 += sm->res[((2 * lane) * S::KC1 + c) * MM + m];
            v1 += sm->res[((2 * lane + 1) * S::KC1 + c) * MM + m];
          }
          put_granule(gg + ((size_t)m * 2 * H + n1 / 2) * 8, tag,
                      pack_bf16x2(gelu_bloom(v0 + bf16_lo(b1)), gelu_bloom(v1 + bf16_hi(b1))));
        }
      }
    }
    ESTAMP(l, 3, 4);
    // ---------------- E: fc2 -> x2 = x1 + fc2(g) + bias
    bar(); bar();  // S2, S3
    {
      KArgs* A = fresh(a);
      char* gx2 = A->ws + WO::GX2;
      float* out = A->x_out;
      const bool last = l + 1 == L;
      const uint32_t tag = tag_of(st.gen, L, l, E_X2);
      if (lane < S::R2) {
#pragma unroll
        for (int m = 0; m < MM; m++) {
          float v = 0.f;
#pragma unroll
          for (int c = 0; c < S::KC2; c++) v += sm->res[(lane * S::KC2 + c) * MM + m];
          const float y = (v + bf16_lo(b2)) + sm->xf[m * H + n2];
          if (last) out[(size_t)m * H + n2] = y;  // the stage output: read after the launch
          else put_granule(gx2 + ((size_t)m * H + n2) * 8, tag, __float_as_uint(y));
        }
      }
    }
    ESTAMP(l, 4, 4);
  }
  // The block whose publisher finishes last advances the launch counter for the next launch's epochs
  // and resets the control words (the launch's timeout word is kept in STATUS_LAST for
  // bs_engine_status).  Every other block has then published everything; its wave 0 may still be
  // finishing a sweep of this launch, which reads no control word but `status`, set before any block
  // can finish (a timeout makes its own block late, not this one).
  {
    unsigned* ctl = (unsigned*)fresh(a)->ws;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add((gu32*)(ctl + Ctl::DONE), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old == (unsigned)(kG - 1) && lane == 0) {
      st4_sc1(ctl + Ctl::STATUS_LAST, ld4_sc1(ctl + Ctl::STATUS));
      st4_sc1(ctl + Ctl::STATUS, 0u);
      st4_sc1(ctl + Ctl::GEN, st.gen + 1u);
      st4_sc1(ctl + Ctl::DONE, 0u);
    }
  }
#ifdef BS_ENGINE_STAMPS
  for (int i = lane; i < 64 * 5 * 6; i += 64) {  // wave 1's stamps
    const int k = i % 6, ph = (i / 6) % 5;
    if (ph == 1 ? k >= 2 : k == 4) g_eng_stamps[(size_t)blockIdx.x * 64 * 5 * 6 + i] = sm->stamps[i];
  }
#endif
}

template <int MM, int H>
__global__ __launch_bounds__(kThreads) void decode_engine_kernel(EngineArgs a) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ka = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  if (wv >= kIO) role_compute<MM, H>(ka);
  else if (wv == 0) role_io<MM, H>(ka);
  else if (wv == 1) role_pub<MM, H>(ka);
  else role_attn<MM, H>(ka);
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
size_t engine_ws_bytes(int h, int n_head) {
  return 256 + (size_t)96 * h + (size_t)n_head * kMaxSplit * 2 * kRec * 8;  // WsOff<H>::GPART + records
}
size_t engine_layer_bytes(int h) { return h == 1536 ? LayerOff<1536>::END : LayerOff<1024>::END; }
size_t engine_status_offset() { return (size_t)Ctl::STATUS_LAST * 4; }

static int engine_device_ok(int device) {
  static int cached[64];
  static bool init[64];
  if (device < 0 || device >= 64) return 0;
  if (!init[device]) {
    hipDeviceProp_t p;
    int ok = hipGetDeviceProperties(&p, device) == hipSuccess && p.multiProcessorCount >= kG;
    if (ok) {
      int nb = 0;
      ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, decode_engine_kernel<2, 1536>, kThreads,
                                                        sizeof(Smem<2, 1536>)) == hipSuccess &&
           nb >= 1;
    }
    cached[device] = ok;
    init[device] = true;
  }
  return cached[device];
}

bool engine_supported(int device, int M, int h, int n_head, int max_ctx) {
  if (M < 1 || M > 2) return false;
  if (h != 1024 && h != 1536) return false;
  const int hd = h / n_head;
  if (h % n_head || hd % 8 || hd > 128 || hd < 16) return false;
  const int pb = 64 / M, ns = (max_ctx + pb - 1) / pb;  // AttnGeom<M>::PB
  if (n_head * ns > kG || ns > kMaxSplit) return false;  // attention blocks within the grid
  return engine_device_ok(device) != 0;
}

void launch_decode_engine(const EngineArgs& a, hipStream_t s) {
  const int H = a.h;
  if (a.M == 1) {
    if (H == 1536) decode_engine_kernel<1, 1536><<<kG, kThreads, sizeof(Smem<1, 1536>), s>>>(a);
    else decode_engine_kernel<1, 1024><<<kG, kThreads, sizeof(Smem<1, 1024>), s>>>(a);
  } else {
    if (H == 1536) decode_engine_kernel<2, 1536><<<kG, kThreads, sizeof(Smem<2, 1536>), s>>>(a);
    else decode_engine_kernel<2, 1024><<<kG, kThreads, sizeof(Smem<2, 1024>), s>>>(a);
  }
}
