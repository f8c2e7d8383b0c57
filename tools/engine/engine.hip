// tools/engine/engine.hip — the persistent decode engine: every decoder block of a stage for one decode step of
// ONE row (S = 1, M = 1, bf16, hidden 1024 / 1536, 16 heads) in one launch on gfx950.
// NOT part of the library: measured at parity with the five-launch decode path at best
// (profiles/r04_engine_timeline_ab.txt), it was moved out in round 4 and is kept as the A/B experiment that
// tools/engine_timeline.hip builds (the stage's host integration and parity tests were removed with it; the
// last library version with them is in git history).
//
// Why: at batch 1 a bloom-1b1 layer is five dependent weight-streaming launches (LN+QKV 5.4, attention 4.8,
// dense 4.8, LN+fc1 5.4, fc2 5.1 us) moving 56.6 MB -- 8.7 us of HBM streaming at 6.5 TB/s; the rest is kernel
// boundaries, first-byte latency and drain tails.  The weights do not depend on the activations, so here one
// workgroup per CU streams its share of every layer into an LDS ring AHEAD of the dependency edges, and each
// phase only waits for its activation vector; its dot products then read the weights from LDS.
//
// Round 4 rebuild to MI355X_MICROARCH.md's batch-1 engine recipe ("engine-vs-launches", "ldsdma-fill",
// "nt-weights", "prefetch-credit", "handoff-1to1", "gather-pass", "polling-cost"); round 3's engine streamed the
// weights through a register ring on 12 compute waves, which put every hand-off behind a full memory queue
// (2-4 us per edge, 32.8 us per layer: profiles/r03_engine_timeline.txt).  Per workgroup (256 threads):
//   wave 0  LOADER: the only wave that streams weights -- LDS-DMA (buffer_load ... lds, nt) of the block's rows
//           of every layer, in use order, into a ring of NS slots (one slot = one 2H-byte weight row of QKV /
//           dense / fc1, a quarter row of fc2); at most D slots in flight; `landed` in LDS; a slot is free once
//           every dot wave has moved past its row (per-wave `need` words: the ring refills row by row).
//   wave 1  GATHER: every all-to-all hand-off (x, ctx, x1, g: granule sweeps) and the LayerNorms; stages each
//           phase's input vector in LDS.
//   wave 2  ATTENTION: the block's (head, context split): the head's new q/k/v gathered, the split's cached K/V
//           rows (landed in LDS by the loader), one (max, sum, acc) record from three partials (waves 2, 1, 3 each
//           take a third of the rows); the head's split-0 block merges the 16 records into ctx.
//   wave 3  PUBLISH: every epilogue (bias, residual, GELU, KV-cache row) and every global store.
//   Dot products of every phase: rows split over waves 1-3 (v_dot2 on LDS weights x registered activations).
// Loads and stores live on different waves: a wave with write-through stores pending would wait for them
// before using any later load (the compiler's vmcnt is in order).
//
// Placement: block b owns QKV rows [b RQ, (b+1) RQ) -- with HF's per-head [3][hd] interleave that is head
// h = b / 16's rows -- and does that head's attention over context split s = b % 16, so the q/k/v and record
// hand-offs stay inside a 16-block head group; dense / fc1 / fc2 rows are contiguous per block.
//
// Per layer l: A x -> LN_in -> QKV rows -> q/k/v granules, KV cache | B attention record -> merge (s = 0) ->
// ctx granules | C ctx -> dense + bias + x -> x1 | D x1 -> LN_post -> fc1 + bias, GELU -> g | E g -> fc2 + bias
// + x1 -> x (next layer's input, or the stage output).
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", R2: the data is the flag): each value travels as an 8-byte
// granule {value, tag} written by ONE sc1 store; consumers re-read with 16-B sc1 loads until every tag equals
// the edge's epoch 0x80000000 | ((gen * L + l) * 8 + edge), `gen` = a launch counter the last block advances,
// so no buffer is ever cleared.  Every spin is bounded (200 ms): on expiry the block marks itself dead (every
// later wait falls through, the grid drains), ORs 1 into the stage's sticky error word (host-mapped, never
// reset: bs_forward refuses to run once it is set) and the step's outputs are garbage.  The grid assumes all
// 256 workgroups resident: the stage refuses the engine inside a multi-rank pipeline (RCCL kernels hold CUs).
#include "../../distributed_inference_demo_amd/csrc/common.h"
#include "../../distributed_inference_demo_amd/csrc/kernels.h"

// ---- Persistent decode engine: every decoder block of a bf16 stage for one decode step
// (S = 1, one row, hidden 1024 / 1536, 16 heads, contexts <= 1024) in one launch of one workgroup per CU; an
// LDS-DMA loader wave streams the block's weights ahead of the dependency edges.  Layer l's tensor t is at
// (layer-0 pointer) + l * layer_stride bytes.
struct EngineArgs {
  const char* wl;          // layer 0's tensors (arena order, engine.hip LayerOff); layer l at + l * layer_stride
  size_t layer_stride;
  const char* kv;          // KV cache of layer 0: K at kv, V at kv + kv_half; layer l at + l * kv_layer_stride
  size_t kv_layer_stride, kv_half;
  int L, M, h, n_head, hd, max_ctx, slot;
  float eps, inv_norm;
  const float* slopes;     // [n_head]
  const int* past_dev;     // [M] cached length of each row
  const float* x_in;       // [M][h] fp32 stage input, or null on the first stage:
  const int* ids;          //   token ids [M] -> word_embeddings + word_embeddings_layernorm
  const void *wemb, *emb_g, *emb_b;
  float* x_out;            // [M][h] fp32 stage output (residual stream after the last block)
  char* ws;                // engine_ws_bytes(h, n_head), zeroed once at init: control words + granule buffers
  unsigned* sticky_host;   // host-mapped error word: 1 once any in-kernel wait expired (never reset)
};
size_t engine_status_offset();  // byte offset in EngineArgs::ws of the sticky timeout word
size_t engine_ws_bytes(int h, int n_head);
size_t engine_layer_bytes(int h);  // bytes of one layer's tensors in the arena (the offsets the kernel assumes)
bool engine_supported(int device, int M, int h, int n_head, int max_ctx);
void launch_decode_engine(const EngineArgs& a, hipStream_t s);

namespace {

constexpr int kG = 256, kThreads = 256, kNH = 16, kSplits = 16;
// Build knobs for tools/engine_timeline.hip's A/B binaries (the product library uses the defaults):
// BS_ENGINE_D slots in flight per CU; BS_ENGINE_THIN = T > 0 holds the loader to T outstanding slots while the
// CU's gather wave sweeps a hand-off (MI355X_MICROARCH.md "gather-pass").
#ifndef BS_ENGINE_D
#define BS_ENGINE_D 8
#endif
#ifndef BS_ENGINE_THIN
#define BS_ENGINE_THIN 0
#endif
constexpr int kD = BS_ENGINE_D;                          // weight slots in flight per CU (loader)
constexpr int kMaxPos = 64;                             // cached positions per attention split (contexts <= 1024)
enum Edge { E_X = 0, E_QKV = 1, E_PART = 2, E_CTX = 3, E_X1 = 4, E_G = 5 };
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms of s_memrealtime (100 MHz)

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
}
// 16-B sc1 load (L1 bypass): two granules another workgroup published in this launch
__device__ __forceinline__ u32x4v ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
// one granule {value, tag}: ONE aligned 8-byte sc1 store
__device__ __forceinline__ void put_granule(void* p, uint32_t tag, uint32_t value) {
  __hip_atomic_store((gu64*)p, ((unsigned long long)tag << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t tag_of(uint32_t gen, int L, int l, int e) {
  return 0x80000000u | (((gen * (uint32_t)L + (uint32_t)l) * 8u + (uint32_t)e) & 0x7FFFFFFFu);
}
typedef float f2v __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_add / v_pk_mul / v_pk_fma_f32)
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{a, b}, bf2v));
}
__device__ __forceinline__ float bf16_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t v) { return __uint_as_float(v & 0xFFFF0000u); }
__device__ __forceinline__ float bf16_at(const void* p, int i) {
  return __uint_as_float((uint32_t)((const unsigned short*)p)[i] << 16);
}

// LDS words shared by the waves (workgroup-scope atomics: never cached in registers)
__device__ __forceinline__ int lds_get(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_put(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS data writes land before the flag
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The loader's publish of `landed`: an inline-asm ds_write, which the compiler does not see as an LDS access
// -- for a visible one it drains the wave's LDS-DMA first (vmcnt(0): it cannot tell the ring from the word),
// which held the loader to one slot in flight (4 GB/s per CU, round-4 first timeline).  The explicit counted
// vmcnt before it is what orders the landed slots.
__device__ __forceinline__ void lds_put_loader(uint32_t off, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(off), "v"(v));
}
// An LDS word read the compiler does not see either (the loader polls att_ready with it between LDS-DMA
// issues without draining them).
__device__ __forceinline__ int lds_peek_loader(uint32_t off) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(off));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void lds_add(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Layer tensors: one arena, every tensor 256-B aligned in canonical order (stage.hip init_stage); for
// h % 128 == 0 every size is a multiple of 256 B, so the offsets inside a layer are constants of H.
template <int H> struct LayerOff {
  static constexpr size_t LN1_G = 0, LN1_B = LN1_G + 2 * H, QKV_W = LN1_B + 2 * H, QKV_B = QKV_W + 6ull * H * H,
                          DENSE_W = QKV_B + 6 * H, DENSE_B = DENSE_W + 2ull * H * H, LN2_G = DENSE_B + 2 * H,
                          LN2_B = LN2_G + 2 * H, FC1_W = LN2_B + 2 * H, FC1_B = FC1_W + 8ull * H * H,
                          FC2_W = FC1_B + 8 * H, FC2_B = FC2_W + 8ull * H * H, END = FC2_B + 2 * H;
};

template <int H> struct Cfg {
  static constexpr int HD = H / kNH, REC = HD + 2;                   // head dim; split record (max, sum, acc)
  static constexpr int NC = H / 512;                                  // 1-KB pieces of a 2H-byte row
  static constexpr int RQ = 3 * H / kG, RD = H / kG, R1 = 4 * H / kG, R2 = H / kG;  // rows per block
  static constexpr int SQ = RQ, SD = RD, S1 = R1, S2 = 4 * R2;       // ring slots per phase (slot = 2H bytes)
  static constexpr int OQ = 0, OD = SQ, O1 = SQ + SD, O2 = SQ + SD + S1, SL = SQ + SD + S1 + S2;
  // ring slots: what the 160 KB of LDS holds beside the rest of Smem (with the diagnostic stamps)
  static constexpr int SLOT = 2 * H, NS = H == 1536 ? 35 : 60, RING = NS * SLOT;
  static_assert(NS >= S1 && NS >= S2 && NS >= SQ, "a phase's slots fit the ring");
  static_assert(kD * NC <= 63, "vmcnt immediate");
};

// Workspace (EngineArgs::ws, zeroed at init): control words, then granule buffers.
struct Ctl { static constexpr int GEN = 0, DONE = 16, STICKY = 32; };
template <int H> struct WsOff {
  using C = Cfg<H>;
  static constexpr size_t GX = 256, GX1 = GX + 8 * H, GQKV = GX1 + 8 * H, GCTX = GQKV + 12 * H, GG = GCTX + 4 * H,
                          GPART = GG + 16 * H, END = GPART + (size_t)kNH * kSplits * C::REC * 8;
};

template <int H> struct Smem {
  using C = Cfg<H>;
  alignas(16) char ring[C::RING];                     // weight slots (LDS-DMA destination)
  alignas(16) bf16 xa[2][H];                          // phase inputs: LN_in out / ctx (A, C: 0 / 1), LN_post out (D: 0)
  alignas(16) bf16 xg[4 * H];                         // phase E input: g
  alignas(16) float xf[C::RD];                        // the block's residual rows (dense = fc2 rows): x during A..C, x1 during D..E
  alignas(16) bf16 kv[2][kMaxPos][C::HD];             // attention: this split's cached K and V rows
  alignas(16) float mg[kSplits][C::REC];              // attention: the 3 partials, then the merge (split 0): the head's records
  alignas(16) float pr[kMaxPos];                      // attention: probabilities
  alignas(16) float rec[C::REC];                      // attention: this split's record
  alignas(16) bf16 qkv[3][C::HD];                     // attention: the head's q, k, v of the new position
  alignas(16) bf16 ctxh[C::HD];                       // attention merge: the head's context
  alignas(16) float res[32];                          // dot results of the phase's rows
  int landed, dots_done, in_ready, att_ready, merge_ready, dead, gathering, qkv_ready, att_parts;
  int need[3];                                        // per dot wave: the first slot it may still read
#ifdef BS_ENGINE_STAMPS
  unsigned long long stamps[24][16];                  // diagnostic builds: s_memrealtime per (layer, point)
#endif
};

static_assert(sizeof(Smem<1536>) <= 163840 && sizeof(Smem<1024>) <= 163840, "one workgroup's LDS");
static_assert(Cfg<1536>::RD == Cfg<1536>::R2 && Cfg<1024>::RD == Cfg<1024>::R2, "xf holds the dense = fc2 rows");

}  // namespace

// Diagnostic builds only (tools/engine_timeline.hip defines BS_ENGINE_STAMPS): lane 0 of a wave records
// s_memrealtime (100 MHz) at point k of layer l in LDS; the block copies them out at the end.  Points:
// gather wave 0 x seen, 1 LN_in staged, 2 ctx seen, 3 x1 seen, 4 g seen; attention wave 5 q/k/v seen,
// 6 record ready, 7 merged (split 0); publish wave 8 QKV dots done, 9 q/k/v published, 10 record published,
// 11 ctx published (split 0), 12 x1 published, 13 g published, 14 x published; loader 15 layer issued.
#ifdef BS_ENGINE_STAMPS
__device__ unsigned long long g_eng_stamps[256 * 24 * 16];
#define ESTAMP(l, k)                                                                                  \
  do {                                                                                                \
    if ((threadIdx.x & 63) == 0 && (l) < 24) sm->stamps[l][k] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#else
#define ESTAMP(l, k) do {} while (0)
#endif

typedef const __attribute__((address_space(4))) EngineArgs KArgs;  // kernarg segment: scalar loads
__device__ __forceinline__ KArgs* kargs(uint64_t bits) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bits), hi = __builtin_amdgcn_readfirstlane((uint32_t)(bits >> 32));
  return (KArgs*)(((uint64_t)hi << 32) | lo);
}
extern __shared__ __attribute__((aligned(16))) char engine_lds[];
template <int H> __device__ __forceinline__ Smem<H>* smem() { return (Smem<H>*)engine_lds; }

// Expiry of a bounded wait: mark the block dead (every later wait falls through) and set the sticky words.
template <int H>
__device__ __noinline__ void expire(KArgs* a, Smem<H>* sm) {
  __hip_atomic_store(&sm->dead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or((gu32*)((unsigned*)a->ws + Ctl::STICKY), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a->sticky_host) __hip_atomic_fetch_or(a->sticky_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait until LDS word *p >= v (one lane polls with s_sleep: MI355X_MICROARCH.md "polling-cost").
template <int H>
__device__ __forceinline__ void wait_ge(KArgs* a, Smem<H>* sm, int* p, int v) {
  if (lds_get(p) >= v) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (lds_get(p) < v) {
    if (lds_get(&sm->dead)) return;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { expire<H>(a, sm); return; }
  }
}

// Wave-uniform bounded sweep: pairs p = c * 64 + lane (c < NC, p < npairs) of two granules each, at byte
// offset off(p) in r, re-read until every tag equals `tag`; then v[c] = (value0, value1).
template <int H, int NC, typename OFF>
__device__ void sweep(KArgs* a, Smem<H>* sm, __amdgpu_buffer_rsrc_t r, int npairs, OFF off, uint32_t tag,
                      uint32_t (&v)[NC][2]) {
  const int lane = threadIdx.x & 63;
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
    if (__all(ok) || lds_get(&sm->dead)) return;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { if (lane == 0) expire<H>(a, sm); return; }
  }
}

// A row's LayerNorm (nn.LayerNorm: two-pass mean / biased variance, eps inside the sqrt) over the NP value
// pairs each lane holds (elements (c * 64 + lane) * 2 + {0, 1}).
template <int NP>
__device__ __forceinline__ void ln_pairs(float (&v)[NP][2], float eps, int n) {
  // one wave does a whole row: packed fp32 halves its VALU issue (the LayerNorm is issue-bound, ~4 cycles
  // per wave64 instruction)
  f2v s = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NP; c++) s += f2v{v[c][0], v[c][1]};
  const float mean = wave_sum(s.x + s.y) / (float)n;
  const f2v m2 = {mean, mean};
  f2v q = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NP; c++) {
    const f2v d = f2v{v[c][0], v[c][1]} - m2;
    q = __builtin_elementwise_fma(d, d, q);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q.x + q.y) / (float)n + eps);
  const f2v r2 = {rstd, rstd};
#pragma unroll
  for (int c = 0; c < NP; c++) {
    const f2v t = (f2v{v[c][0], v[c][1]} - m2) * r2;
    v[c][0] = t.x; v[c][1] = t.y;
  }
}

// ============ wave 0: the weight loader
// Slot g of the launch = ring position g % NS; layer g / SL, phase slot g % SL (OQ.., OD.., O1.., O2..).
template <int H>
__device__ __attribute__((noinline)) void role_loader(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<H>* sm = smem<H>();
  using C = Cfg<H>;
  using LO = LayerOff<H>;
  const int lane = threadIdx.x & 63, b = blockIdx.x;
  const int L = a->L, total = L * C::SL;
  const size_t ls = a->layer_stride;
  auto src = [&](int i) -> uint32_t {  // byte offset of phase slot i inside the layer (+ this lane's 16 B)
    size_t o;
    if (i < C::OD) o = LO::QKV_W + (size_t)(b * C::RQ + i) * C::SLOT;
    else if (i < C::O1) o = LO::DENSE_W + (size_t)(b * C::RD + (i - C::OD)) * C::SLOT;
    else if (i < C::O2) o = LO::FC1_W + (size_t)(b * C::R1 + (i - C::O1)) * C::SLOT;
    else o = LO::FC2_W + (size_t)b * C::R2 * 4 * C::SLOT + (size_t)(i - C::O2) * C::SLOT;
    return (uint32_t)o + lane * 16;
  };
  // Everything the steady loop needs lives in registers: the asm waits below clobber "memory", which would
  // otherwise re-load the LDS base (a table lookup in a non-kernel function) and the kernel arguments per slot.
  uint32_t ring0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)sm->ring;
  uint32_t landed_off = (uint32_t)(size_t)(__attribute__((address_space(3))) int*)&sm->landed;
  uint32_t att_off = (uint32_t)(size_t)(__attribute__((address_space(3))) int*)&sm->att_ready;
  uint32_t kv_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)&sm->kv[0][0][0];
  const char* wl0 = a->wl;
  // this block's attention split (wave 2's head and positions): its cached K / V rows are contiguous
  // [ncache][HD] in the cache and land in sm->kv by LDS-DMA ahead of each layer's QKV slots
  constexpr int HD = C::HD, NKV = kMaxPos * HD * 2 / 1024;
  const int head = b / kSplits, s = b % kSplits, past = a->past_dev[0];
  const int per = (past + 1 + kSplits - 1) / kSplits, p0 = s * per;
  const int ncache = max(0, min(p0 + per, past) - p0);
  const int kvbytes = ncache * HD * 2;
  const char* kv0 = a->kv + ((size_t)a->slot * kNH + head) * a->max_ctx * HD * 2 + (size_t)(ncache > 0 ? p0 : 0) * HD * 2;
  uint32_t gath_off = (uint32_t)(size_t)(__attribute__((address_space(3))) int*)&sm->gathering;
  asm volatile("" : "+s"(ring0), "+s"(landed_off), "+s"(att_off), "+s"(kv_lds), "+s"(wl0), "+s"(kv0), "+s"(gath_off));
  int pub = 0;  // landed as published: monotone (the ring-full and thinned paths publish ahead of the counted one)
  auto publish = [&](int v) {
    if (v > pub) { pub = v; lds_put_loader(landed_off, v); }
  };
  int freed = 0;
  for (int g = 0; g < total; g++) {
    if (g - freed >= C::NS) {
      // the ring is full: everything issued lands first (consumers may be waiting for it), then wait for room
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      publish(g);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        freed = min(lds_get(&sm->need[0]), min(lds_get(&sm->need[1]), lds_get(&sm->need[2])));
        if (g - freed < C::NS || lds_get(&sm->dead)) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { expire<H>(a, sm); break; }
      }
      if (lds_get(&sm->dead)) break;
    }
    if (BS_ENGINE_THIN && lds_peek_loader(gath_off)) {
      // the gather wave is sweeping: at most BS_ENGINE_THIN slots in flight (this one included), so its loads
      // do not queue behind a refill burst (MI355X_MICROARCH.md "gather-pass")
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((BS_ENGINE_THIN - 1) * C::NC) : "memory");
      publish(g - BS_ENGINE_THIN + 1);
    }
    const int l = g / C::SL, i = g - l * C::SL;
    if (i == 0 && kvbytes > 0) {
      // layer l's K / V rows of the split, once the attention wave is done with layer l - 1's; loads return
      // in order, so they have landed once slot g + 1 has (the attention wave's first QKV row waits for it)
      if (l > 0 && lds_peek_loader(att_off) < l) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (lds_peek_loader(att_off) < l) {
          if (lds_get(&sm->dead)) break;
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { expire<H>(a, sm); break; }
        }
      }
      const char* kl = kv0 + (size_t)l * a->kv_layer_stride;
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(kl), (short)0, kvbytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(kl + a->kv_half), (short)0, kvbytes, 0x00020000);
#pragma unroll
      for (int c = 0; c < NKV; c++) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(size_t)(kv_lds + c * 1024), 16, c * 1024 + lane * 16, 0, 0, 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void*)(size_t)(kv_lds + kMaxPos * HD * 2 + c * 1024), 16,
                                                 c * 1024 + lane * 16, 0, 0, 2);
      }
    }
    const __amdgpu_buffer_rsrc_t r = rsrc(wl0 + (size_t)l * ls);
    const uint32_t so = src(i);
    const uint32_t dst = ring0 + (uint32_t)((g % C::NS) * C::SLOT);
#pragma unroll
    for (int p = 0; p < C::NC; p++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(size_t)(dst + p * 1024), 16, so + p * 1024, 0, 0, 2 /* nt */);
    // at most kD slots in flight: slot g - kD + 1 has landed once all but the youngest (kD - 1) * NC have
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kD - 1) * C::NC) : "memory");
    publish(g - kD + 2);
#ifdef BS_ENGINE_STAMPS
    if (i == C::SL - 1 && l < 24 && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      asm volatile("ds_write_b64 %0, %1" ::"v"(landed_off + (uint32_t)((char*)&sm->stamps[l][15] - (char*)&sm->landed)),
                   "v"(t));
    }
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_put(&sm->landed, total);
}

// ============ dot products of phase (l, k): rows j = wc, wc + 3, ... of the block's nrows rows, each SPR slots
// long, against the phase input x (bf16, K = SPR * H elements) staged in LDS.  Every dot wave then adds one
// to dots_done.
template <int H, int SPR>
__device__ __forceinline__ void phase_dots(KArgs* a, Smem<H>* sm, int wc, int g0, int nrows, int P, const bf16* x) {
  using C = Cfg<H>;
  constexpr int NCK = SPR * C::NC;  // 512-element chunks of a row
  const int lane = threadIdx.x & 63;
  wait_ge<H>(a, sm, &sm->in_ready, P + 1);
  bf16x8 xr[NCK];
#pragma unroll
  for (int c = 0; c < NCK; c++) xr[c] = *reinterpret_cast<const bf16x8*>(x + c * 512 + lane * 8);
  for (int j = wc; j < nrows; j += 3) {
    wait_ge<H>(a, sm, &sm->landed, g0 + (j + 1) * SPR);
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < NCK; c++) {
      const int g = g0 + j * SPR + c / C::NC;
      const bf16x8 w = *reinterpret_cast<const bf16x8*>(sm->ring + (g % C::NS) * C::SLOT + (c % C::NC) * 1024 + lane * 16);
      acc = dot8(w, xr[c], acc);
    }
    const float v = wave_sum(acc);
    if (lane == 0) {
      sm->res[j] = v;
      // this wave's next row (or the phase end): every slot before it is read -- the loader may refill it
      lds_put(&sm->need[wc], g0 + min(j + 3, nrows) * SPR);
    }
  }
  if (lane == 0) lds_add(&sm->dots_done, 1);
}

// ============ one third of the split's attention: rows j of passes [q pp, (q + 1) pp) (4 rows per pass, 16 lanes
// per row, 8 dims each -- every LDS read a contiguous 16-B chunk of one row) -> the partial (max, sum, acc) in
// mg[q] (the merge area is free until the record edge).  Waves 2, 1 and 3 take parts 0, 1, 2: the attention is
// issue-bound on one wave (~4 cycles per wave64 instruction), and waves 1 and 3 would otherwise wait.
// Row j < ncache is a cached row (sm->kv), j == ncache (position `past`) the new k / v, rows past npos masked.
template <int H>
__device__ __forceinline__ void attn_part(Smem<H>* sm, int q, int p0, int npos, int ncache, float slope, float inv_norm) {
  using C = Cfg<H>;
  constexpr int HD = C::HD, NSL = HD / 8;
  const int lane = threadIdx.x & 63, grp = lane >> 4, ds = lane & 15;
  const bool dv = ds < NSL;
  const int doff = dv ? ds * 8 : 0;
  const int npass = (npos + 3) / 4, pp = (npass + 2) / 3;  // passes <= kMaxPos / 4
  const int t0 = min(q * pp, npass), t1 = min(t0 + pp, npass);
  const bf16x8 q8 = *reinterpret_cast<const bf16x8*>(sm->qkv[0] + doff);
  float mx = -INFINITY;
  for (int t = t0; t < t1; t += 4) {
    bf16x8 kk[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = min((t + u) * 4 + grp, kMaxPos - 1);
      kk[u] = *reinterpret_cast<const bf16x8*>((j < ncache ? sm->kv[0][j] : sm->qkv[1]) + doff);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = (t + u) * 4 + grp;
      float d = dot8(kk[u], q8, 0.f);
      d = dv ? d : 0.f;
      d += dpp_f<0xB1>(d);   // sum over the row's 16 lanes: xor 1, xor 2, rotate 4, rotate 8
      d += dpp_f<0x4E>(d);
      d += dpp_f<0x124>(d);
      d += dpp_f<0x128>(d);
      const bool mine = t + u < t1;
      const float sc = mine && j < npos ? slope * (float)(p0 + j) + inv_norm * d : -INFINITY;
      if (ds == 0 && mine) sm->pr[j] = sc;
      mx = fmaxf(mx, sc);
    }
  }
  mx = wave_max(mx);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // fp32 softmax partial: lane i <-> row 4 t0 + i
  const int jr = 4 * t0 + lane;
  const bool own = lane < 4 * (t1 - t0) && jr < npos;
  const float e = own ? __expf(sm->pr[min(jr, kMaxPos - 1)] - mx) : 0.f;
  const float lsum = wave_sum(e);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (own) sm->pr[jr] = e;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = 0.f;
  for (int t = t0; t < t1; t += 4) {
    bf16x8 vv[4];
    float pj[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = min((t + u) * 4 + grp, kMaxPos - 1);
      vv[u] = *reinterpret_cast<const bf16x8*>((j < ncache ? sm->kv[1][j] : sm->qkv[2]) + doff);
      pj[u] = sm->pr[j];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = (t + u) * 4 + grp;
      const float w = t + u < t1 && j < npos ? pj[u] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; k++) acc[k] += w * (float)vv[u][k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    acc[k] += __shfl_xor(acc[k], 16, 64);
    acc[k] += __shfl_xor(acc[k], 32, 64);
  }
  if (grp == 0 && dv) {
#pragma unroll
    for (int k = 0; k < 8; k++) sm->mg[q][2 + doff + k] = acc[k];
  }
  if (lane == 0) { sm->mg[q][0] = mx; sm->mg[q][1] = lsum; }
}

// The block's attention split: positions [p0, p0 + npos), ncache of them cached.
__device__ __forceinline__ void attn_split(KArgs* a, int b, int& p0, int& npos, int& ncache) {
  const int past = a->past_dev[0], s = b % kSplits;
  const int per = (past + 1 + kSplits - 1) / kSplits;  // positions per split (<= kMaxPos)
  p0 = s * per;
  const int p1 = min(p0 + per, past + 1);
  ncache = max(0, min(p1, past) - p0);
  npos = max(0, p1 - p0);
}

// ============ wave 1: the all-to-all gathers and the LayerNorms; stages each phase's input
template <int H>
__device__ __attribute__((noinline)) void role_gather(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<H>* sm = smem<H>();
  using C = Cfg<H>;
  using LO = LayerOff<H>;
  using WO = WsOff<H>;
  constexpr int NP = H / 128;  // fp32 granule pairs per lane of an H-vector
  const int lane = threadIdx.x & 63;
  const int L = a->L;
  const size_t ls = a->layer_stride;
  const uint32_t gen = __builtin_amdgcn_readfirstlane(((const unsigned*)a->ws)[Ctl::GEN]);
  int ap0, anpos, ancache;
  attn_split(a, blockIdx.x, ap0, anpos, ancache);
  float aslope = a->slopes[blockIdx.x / kSplits], ainv = a->inv_norm;
  asm volatile("" : "+v"(aslope), "+v"(ainv));
  // fp32 granule vector (x, x1): v[c] = elements (c * 64 + lane) * 2 + {0, 1}
  auto gather_f32 = [&](size_t off, uint32_t tag, float (&v)[NP][2]) {
    uint32_t raw[NP][2];
    if (BS_ENGINE_THIN) lds_put(&sm->gathering, 1);
    sweep<H, NP>(a, sm, rsrc(a->ws + off), H / 2, [&](int p) { return (uint32_t)(p * 16); }, tag, raw);
    if (BS_ENGINE_THIN) lds_put(&sm->gathering, 0);
#pragma unroll
    for (int c = 0; c < NP; c++) { v[c][0] = __uint_as_float(raw[c][0]); v[c][1] = __uint_as_float(raw[c][1]); }
  };
  // bf16-pair granule vector of n elements -> LDS dst (n / 4 16-B loads, issued together)
  auto gather_bf16 = [&](size_t off, int n, uint32_t tag, bf16* dst) {
    constexpr int NCB = H / 64;  // loads per lane for n = 4H
    uint32_t raw[NCB][2];
    const int np = n / 4;
    if (BS_ENGINE_THIN) lds_put(&sm->gathering, 1);
    sweep<H, NCB>(a, sm, rsrc(a->ws + off), np, [&](int p) { return (uint32_t)(p * 16); }, tag, raw);
    if (BS_ENGINE_THIN) lds_put(&sm->gathering, 0);
#pragma unroll
    for (int c = 0; c < NCB; c++) {
      const int p = c * 64 + lane;
      if (p < np) *reinterpret_cast<uint2*>(dst + p * 4) = make_uint2(raw[c][0], raw[c][1]);
    }
  };
  auto load_gb = [&](const bf16* g, const bf16* be, uint32_t (&gb)[NP][2]) {
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      gb[c][0] = *reinterpret_cast<const uint32_t*>(g + k);
      gb[c][1] = *reinterpret_cast<const uint32_t*>(be + k);
    }
  };
  // x (fp32, registers) -> xf (the block's rows); LN(x) * gamma + beta -> xa[0] (bf16)
  const int xbase = blockIdx.x * C::RD;
  auto stage_ln = [&](float (&v)[NP][2], const uint32_t (&gb)[NP][2], float eps) {
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      if ((unsigned)(k - xbase) < (unsigned)C::RD) *reinterpret_cast<float2*>(&sm->xf[k - xbase]) = make_float2(v[c][0], v[c][1]);
    }
    ln_pairs<NP>(v, eps, H);
#pragma unroll
    for (int c = 0; c < NP; c++) {
      const int k = (c * 64 + lane) * 2;
      const f2v y = __builtin_elementwise_fma(f2v{v[c][0], v[c][1]}, f2v{bf16_lo(gb[c][0]), bf16_hi(gb[c][0])},
                                              f2v{bf16_lo(gb[c][1]), bf16_hi(gb[c][1])});
      *reinterpret_cast<uint32_t*>(&sm->xa[0][k]) = pack_bf16x2(y.x, y.y);
    }
  };
  for (int l = 0; l < L; l++) {
    const char* wl = a->wl + (size_t)l * ls;
    const float eps = a->eps;
    const int P0 = l * 4;
    // ---- A: x -> LN_in
    {
      uint32_t gb[NP][2];
      load_gb((const bf16*)(wl + LO::LN1_G), (const bf16*)(wl + LO::LN1_B), gb);
      float v[NP][2];
      if (l > 0) {
        gather_f32(WO::GX, tag_of(gen, L, l - 1, E_X), v);
      } else if (a->x_in) {
#pragma unroll
        for (int c = 0; c < NP; c++) {
          const float2 t = *reinterpret_cast<const float2*>(a->x_in + (c * 64 + lane) * 2);
          v[c][0] = t.x; v[c][1] = t.y;
        }
      } else {
        // first stage: word_embeddings[id] -> word_embeddings_layernorm (fp32) is the residual stream
        const bf16* row = (const bf16*)a->wemb + (size_t)a->ids[0] * H;
#pragma unroll
        for (int c = 0; c < NP; c++) {
          const uint32_t r = *reinterpret_cast<const uint32_t*>(row + (c * 64 + lane) * 2);
          v[c][0] = bf16_lo(r); v[c][1] = bf16_hi(r);
        }
        ln_pairs<NP>(v, eps, H);
#pragma unroll
        for (int c = 0; c < NP; c++) {
          const int k = (c * 64 + lane) * 2;
          const uint32_t g = *reinterpret_cast<const uint32_t*>((const bf16*)a->emb_g + k);
          const uint32_t be = *reinterpret_cast<const uint32_t*>((const bf16*)a->emb_b + k);
          v[c][0] = v[c][0] * bf16_lo(g) + bf16_lo(be);
          v[c][1] = v[c][1] * bf16_hi(g) + bf16_hi(be);
        }
      }
      ESTAMP(l, 0);
      stage_ln(v, gb, eps);
      lds_put(&sm->in_ready, P0 + 1);
      ESTAMP(l, 1);
    }
    phase_dots<H, 1>(a, sm, 0, l * C::SL + C::OQ, C::RQ, P0, sm->xa[0]);
    // ---- B: attention part 1 (the ctx edge cannot arrive before the record edge anyway)
    wait_ge<H>(a, sm, &sm->qkv_ready, l + 1);
    attn_part<H>(sm, 1, ap0, anpos, ancache, aslope, ainv);
    if (lane == 0) lds_add(&sm->att_parts, 1);
    // ---- C: ctx -> xa[1]
    gather_bf16(WO::GCTX, H, tag_of(gen, L, l, E_CTX), sm->xa[1]);
    ESTAMP(l, 2);
    lds_put(&sm->in_ready, P0 + 2);
    phase_dots<H, 1>(a, sm, 0, l * C::SL + C::OD, C::RD, P0 + 1, sm->xa[1]);
    // ---- D: x1 -> xf, LN_post -> xa[0]
    {
      uint32_t gb[NP][2];
      load_gb((const bf16*)(wl + LO::LN2_G), (const bf16*)(wl + LO::LN2_B), gb);
      float v[NP][2];
      gather_f32(WO::GX1, tag_of(gen, L, l, E_X1), v);
      ESTAMP(l, 3);
      stage_ln(v, gb, eps);
      lds_put(&sm->in_ready, P0 + 3);
    }
    phase_dots<H, 1>(a, sm, 0, l * C::SL + C::O1, C::R1, P0 + 2, sm->xa[0]);
    // ---- E: g -> xg
    gather_bf16(WO::GG, 4 * H, tag_of(gen, L, l, E_G), sm->xg);
    ESTAMP(l, 4);
    lds_put(&sm->in_ready, P0 + 4);
    phase_dots<H, 4>(a, sm, 0, l * C::SL + C::O2, C::R2, P0 + 3, sm->xg);
  }
}

// ============ wave 2: attention of the block's (head, split); the head's merge on split 0
template <int H>
__device__ __attribute__((noinline)) void role_attn(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<H>* sm = smem<H>();
  using C = Cfg<H>;
  using WO = WsOff<H>;
  constexpr int HD = C::HD;
  const int lane = threadIdx.x & 63, b = blockIdx.x, head = b / kSplits, s = b % kSplits;
  const int L = a->L, mctx = a->max_ctx;
  const uint32_t gen = __builtin_amdgcn_readfirstlane(((const unsigned*)a->ws)[Ctl::GEN]);
  int p0, npos, ncache;
  attn_split(a, b, p0, npos, ncache);
  float slope = a->slopes[head], inv_norm = a->inv_norm;
  asm volatile("" : "+v"(slope), "+v"(inv_norm));  // held in registers (else re-read from the kernarg per position)
  for (int l = 0; l < L; l++) {
    const int P0 = l * 4;
    // the split's cached K / V rows arrive in sm->kv by the loader's LDS-DMA (issued before this layer's
    // QKV slots: landed once the QKV rows below are)
    phase_dots<H, 1>(a, sm, 1, l * C::SL + C::OQ, C::RQ, P0, sm->xa[0]);
    // the head's new q, k, v (3 HD bf16 = 3 HD / 2 granules)
    {
      constexpr int NQ = (3 * HD / 4 + 63) / 64;
      uint32_t raw[NQ][2];
      sweep<H, NQ>(a, sm, rsrc(a->ws + WO::GQKV), 3 * HD / 4,
                   [&](int p) { return (uint32_t)((head * 3 * HD / 2 + p * 2) * 8); }, tag_of(gen, L, l, E_QKV), raw);
#pragma unroll
      for (int c = 0; c < NQ; c++) {
        const int p = c * 64 + lane;
        if (p < 3 * HD / 4) *reinterpret_cast<uint2*>(&sm->qkv[0][0] + p * 4) = make_uint2(raw[c][0], raw[c][1]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_put(&sm->qkv_ready, l + 1);
    ESTAMP(l, 5);
    attn_part<H>(sm, 0, p0, npos, ncache, slope, inv_norm);
    // the three partials -> this split's record (max, sum, acc)
    wait_ge<H>(a, sm, &sm->att_parts, 2 * (l + 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    {
      const float m0 = sm->mg[0][0], m1 = sm->mg[1][0], m2 = sm->mg[2][0];
      const float M = fmaxf(m0, fmaxf(m1, m2));
      const float w0 = m0 == -INFINITY ? 0.f : __expf(m0 - M), w1 = m1 == -INFINITY ? 0.f : __expf(m1 - M),
                  w2 = m2 == -INFINITY ? 0.f : __expf(m2 - M);
#pragma unroll
      for (int h2 = 0; h2 < 2; h2++) {
        const int d = lane + 64 * h2;
        if (d < HD) sm->rec[2 + d] = w0 * sm->mg[0][2 + d] + w1 * sm->mg[1][2 + d] + w2 * sm->mg[2][2 + d];
      }
      if (lane == 0) {
        sm->rec[0] = npos > 0 ? M : -INFINITY;
        sm->rec[1] = w0 * sm->mg[0][1] + w1 * sm->mg[1][1] + w2 * sm->mg[2][1];
      }
      if (lane == 0) lds_put(&sm->att_ready, l + 1);
      ESTAMP(l, 6);
    }
    if (s == 0) {
      // the head's 16 records -> ctx_h = sum_s w_s acc_s / sum_s w_s l_s, w_s = exp(m_s - max m)
      constexpr int NR = (kSplits * C::REC / 2 + 63) / 64;
      uint32_t raw[NR][2];
      sweep<H, NR>(a, sm, rsrc(a->ws + WO::GPART), kSplits * C::REC / 2,
                   [&](int p) { return (uint32_t)((head * kSplits * C::REC + p * 2) * 8); }, tag_of(gen, L, l, E_PART), raw);
#pragma unroll
      for (int c = 0; c < NR; c++) {
        const int p = c * 64 + lane;
        if (p < kSplits * C::REC / 2) {
          (&sm->mg[0][0])[2 * p] = __uint_as_float(raw[c][0]);
          (&sm->mg[0][0])[2 * p + 1] = __uint_as_float(raw[c][1]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int t = min(lane, kSplits - 1);
      const float mt = sm->mg[t][0], lt = sm->mg[t][1];
      const bool ok = lane < kSplits && mt != -INFINITY;
      const float M = wave_max(ok ? mt : -INFINITY);
      const float w = ok ? __expf(mt - M) : 0.f;
      const float Ls = wave_sum(w * (ok ? lt : 0.f));
      if (lane < kSplits) sm->pr[lane] = w;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int h2 = 0; h2 < 2; h2++) {
        const int d = lane + 64 * h2;
        if (d < HD) {
          float o = 0.f;
          for (int u = 0; u < kSplits; u++) o += sm->pr[u] * sm->mg[u][2 + d];
          sm->ctxh[d] = (bf16)(o / Ls);
        }
      }
      if (lane == 0) lds_put(&sm->merge_ready, l + 1);
      ESTAMP(l, 7);
    }
    phase_dots<H, 1>(a, sm, 1, l * C::SL + C::OD, C::RD, P0 + 1, sm->xa[1]);
    phase_dots<H, 1>(a, sm, 1, l * C::SL + C::O1, C::R1, P0 + 2, sm->xa[0]);
    phase_dots<H, 4>(a, sm, 1, l * C::SL + C::O2, C::R2, P0 + 3, sm->xg);
  }
}

// ============ wave 3: every epilogue and every global store; frees the ring slots of each finished phase
template <int H>
__device__ __attribute__((noinline)) void role_publish(uint64_t ka) {
  KArgs* a = kargs(ka);
  Smem<H>* sm = smem<H>();
  using C = Cfg<H>;
  using LO = LayerOff<H>;
  using WO = WsOff<H>;
  constexpr int HD = C::HD;
  const int lane = threadIdx.x & 63, b = blockIdx.x, head = b / kSplits, s = b % kSplits;
  const int L = a->L, mctx = a->max_ctx, past = a->past_dev[0];
  const size_t ls = a->layer_stride;
  const uint32_t gen = __builtin_amdgcn_readfirstlane(((const unsigned*)a->ws)[Ctl::GEN]);
  char* ws = a->ws;
  int ap0, anpos, ancache;
  attn_split(a, b, ap0, anpos, ancache);
  float aslope = a->slopes[head], ainv = a->inv_norm;
  asm volatile("" : "+v"(aslope), "+v"(ainv));
  // this lane's rows of each epilogue (lanes past a phase's rows compute row 0 and never store)
  const int jq = 2 * min(lane, C::RQ / 2 - 1), jd = min(lane, C::RD - 1), j1 = 2 * min(lane, C::R1 / 2 - 1),
            j2 = min(lane, C::R2 - 1);
  const int nq = b * C::RQ + jq, nd = b * C::RD + jd, n1 = b * C::R1 + j1, n2 = b * C::R2 + j2;
  const int three = 3 * HD, qrr = nq - head * three, qwhich = qrr / HD, qd = qrr - qwhich * HD;
  for (int l = 0; l < L; l++) {
    const char* wl = a->wl + (size_t)l * ls;
    const int P0 = l * 4, g0 = l * C::SL;
    // biases of the layer, requested before any store of it
    const uint32_t bq = *reinterpret_cast<const uint32_t*>((const bf16*)(wl + LO::QKV_B) + nq);
    const uint32_t bd = ((const unsigned short*)(wl + LO::DENSE_B))[nd];
    const uint32_t b1 = *reinterpret_cast<const uint32_t*>((const bf16*)(wl + LO::FC1_B) + n1);
    const uint32_t b2 = ((const unsigned short*)(wl + LO::FC2_B))[n2];
    // ---- A: QKV rows -> q / k / v granules (this step's attention) and k, v to the cache (later steps)
    phase_dots<H, 1>(a, sm, 2, g0 + C::OQ, C::RQ, P0, sm->xa[0]);
    wait_ge<H>(a, sm, &sm->dots_done, 3 * (P0 + 1));
    ESTAMP(l, 8);
    if (lane < C::RQ / 2) {
      const float v0 = sm->res[jq] + bf16_lo(bq), v1 = sm->res[jq + 1] + bf16_hi(bq);
      const uint32_t pk = pack_bf16x2(v0, v1);
      if (qwhich) {
        char* kl = (char*)a->kv + (size_t)l * a->kv_layer_stride + (qwhich == 2 ? a->kv_half : 0);
        *reinterpret_cast<uint32_t*>(kl + ((((size_t)a->slot * kNH + head) * mctx + past) * HD + qd) * 2) = pk;
      }
      put_granule(ws + WO::GQKV + (size_t)(nq / 2) * 8, tag_of(gen, L, l, E_QKV), pk);
    }
    ESTAMP(l, 9);
    // ---- B: attention part 2; this split's record; the head's context (split 0)
    wait_ge<H>(a, sm, &sm->qkv_ready, l + 1);
    attn_part<H>(sm, 2, ap0, anpos, ancache, aslope, ainv);
    if (lane == 0) lds_add(&sm->att_parts, 1);
    wait_ge<H>(a, sm, &sm->att_ready, l + 1);
    {
      const uint32_t tp = tag_of(gen, L, l, E_PART);
      char* rec = ws + WO::GPART + (size_t)(head * kSplits + s) * C::REC * 8;
#pragma unroll
      for (int h2 = 0; h2 < (C::REC + 63) / 64; h2++) {
        const int i = lane + 64 * h2;
        if (i < C::REC) put_granule(rec + i * 8, tp, __float_as_uint(sm->rec[i]));
      }
    }
    ESTAMP(l, 10);
    if (s == 0) {
      wait_ge<H>(a, sm, &sm->merge_ready, l + 1);
      if (2 * lane < HD)
        put_granule(ws + WO::GCTX + (size_t)((head * HD) / 2 + lane) * 8, tag_of(gen, L, l, E_CTX),
                    pack_bf16x2((float)sm->ctxh[2 * lane], (float)sm->ctxh[2 * lane + 1]));
      ESTAMP(l, 11);
    }
    // ---- C: dense -> x1 = x + dense(ctx) + bias
    phase_dots<H, 1>(a, sm, 2, g0 + C::OD, C::RD, P0 + 1, sm->xa[1]);
    wait_ge<H>(a, sm, &sm->dots_done, 3 * (P0 + 2));
    if (lane < C::RD)
      put_granule(ws + WO::GX1 + (size_t)nd * 8, tag_of(gen, L, l, E_X1),
                  __float_as_uint((sm->res[jd] + bf16_lo(bd)) + sm->xf[jd]));
    ESTAMP(l, 12);
    // ---- D: fc1 + bias, GELU -> g
    phase_dots<H, 1>(a, sm, 2, g0 + C::O1, C::R1, P0 + 2, sm->xa[0]);
    wait_ge<H>(a, sm, &sm->dots_done, 3 * (P0 + 3));
    if (lane < C::R1 / 2)
      put_granule(ws + WO::GG + (size_t)(n1 / 2) * 8, tag_of(gen, L, l, E_G),
                  pack_bf16x2(gelu_bloom(sm->res[j1] + bf16_lo(b1)), gelu_bloom(sm->res[j1 + 1] + bf16_hi(b1))));
    ESTAMP(l, 13);
    // ---- E: fc2 -> x = x1 + fc2(g) + bias (the last layer writes the stage output)
    phase_dots<H, 4>(a, sm, 2, g0 + C::O2, C::R2, P0 + 3, sm->xg);
    wait_ge<H>(a, sm, &sm->dots_done, 3 * (P0 + 4));
    if (lane < C::R2) {
      const float y = (sm->res[j2] + bf16_lo(b2)) + sm->xf[j2];
      if (l + 1 == L) a->x_out[n2] = y;
      else put_granule(ws + WO::GX + (size_t)n2 * 8, tag_of(gen, L, l, E_X), __float_as_uint(y));
    }
    ESTAMP(l, 14);
  }
  // The block whose publisher finishes last advances the launch counter for the next launch's epochs.  Every
  // block has then published everything; its other waves may still be reading this launch's granules, which
  // carry this launch's tags (read at kernel start), so the new counter changes nothing for them.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned* ctl = (unsigned*)ws;
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add((gu32*)(ctl + Ctl::DONE), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old == (unsigned)(kG - 1) && lane == 0) {
    __hip_atomic_store((gu32*)(ctl + Ctl::GEN), gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32*)(ctl + Ctl::DONE), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int H>
__global__ __launch_bounds__(kThreads) void decode_engine_kernel(EngineArgs a) {
  Smem<H>* sm = smem<H>();
  if (threadIdx.x == 0) {
    sm->landed = 0; sm->need[0] = 0; sm->need[1] = 0; sm->need[2] = 0; sm->dots_done = 0; sm->in_ready = 0; sm->att_ready = 0; sm->merge_ready = 0;
    sm->dead = 0; sm->gathering = 0; sm->qkv_ready = 0; sm->att_parts = 0;
  }
  __syncthreads();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ka = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  if (wv == 0) role_loader<H>(ka);
  else if (wv == 1) role_gather<H>(ka);
  else if (wv == 2) role_attn<H>(ka);
  else role_publish<H>(ka);
#ifdef BS_ENGINE_STAMPS
  __syncthreads();
  for (int i = threadIdx.x; i < 24 * 16; i += kThreads) g_eng_stamps[(size_t)blockIdx.x * 24 * 16 + i] = (&sm->stamps[0][0])[i];
#endif
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
size_t engine_ws_bytes(int h, int n_head) {
  (void)n_head;
  return h == 1536 ? WsOff<1536>::END : WsOff<1024>::END;
}
size_t engine_layer_bytes(int h) { return h == 1536 ? LayerOff<1536>::END : LayerOff<1024>::END; }
size_t engine_status_offset() { return (size_t)Ctl::STICKY * 4; }

static int engine_device_ok(int device) {
  static int cached[64];
  static bool init[64];
  if (device < 0 || device >= 64) return 0;
  if (!init[device]) {
    hipDeviceProp_t p;
    int ok = hipGetDeviceProperties(&p, device) == hipSuccess && p.multiProcessorCount >= kG;
    if (ok) {
      int nb = 0;
      ok = hipFuncSetAttribute((const void*)decode_engine_kernel<1536>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               sizeof(Smem<1536>)) == hipSuccess &&
           hipFuncSetAttribute((const void*)decode_engine_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               sizeof(Smem<1024>)) == hipSuccess &&
           hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, decode_engine_kernel<1536>, kThreads, sizeof(Smem<1536>)) ==
               hipSuccess &&
           nb >= 1;
    }
    cached[device] = ok;
    init[device] = true;
  }
  return cached[device];
}

bool engine_supported(int device, int M, int h, int n_head, int max_ctx) {
  if (M != 1 || (h != 1024 && h != 1536) || n_head != kNH) return false;
  if (max_ctx > kSplits * kMaxPos) return false;  // every split's cached rows fit the LDS staging
  return engine_device_ok(device) != 0;
}

void launch_decode_engine(const EngineArgs& a, hipStream_t s) {
  if (a.h == 1536) decode_engine_kernel<1536><<<kG, kThreads, sizeof(Smem<1536>), s>>>(a);
  else decode_engine_kernel<1024><<<kG, kThreads, sizeof(Smem<1024>), s>>>(a);
}
