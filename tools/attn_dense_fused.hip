// tools/attn_dense_fused.hip — round 5: split decode attention + the dense GEMV in ONE launch,
// measured against the library's two launches (attn_decode_kernel with deferred merge, then gemv_rows_kernel
// X_PARTS).  Outputs are compared bit for bit; time = 200 back-to-back (attention, dense) pairs between HIP events.
// In the full decode step (bench.py, bloom-1b1 B = 1) the fused launch cost 13 % (profiles/r05_attn_dense_ab.txt):
// every dense block waits on every attention block, an all-to-all in-launch barrier priced at 4-7 us by
// MI355X_MICROARCH.md against ~1.2 us for the kernel boundary it removes.  Kept here, out of the library.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/attn_dense_fused.hip
//        distributed_inference_demo_amd/csrc/attn_prefill.hip -o tools/attn_dense_fused
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <cstdio>
#include <vector>

// ------------------------------------------------------------------------------------
// Split decode attention + the dense GEMV in ONE launch (B <= 2, bf16).  Blocks [0, n_attn) are the
// attention's (head, row, split) blocks (attn_decode_block, 8 waves x 32 positions); each publishes its
// partial sc1 and adds 1 to sync[0].  Blocks [n_attn, n_attn + n_dense) are 8-wave rows-GEMV blocks
// (gemv_rows_block, X_PARTS): they issue their first U weight chunks, one lane polls sync[0] up to n_attn,
// the block merges the partials (sc1 loads) into LDS and streams the rest of the rows.  The dense weights
// are in flight while the attention runs, and the kernel boundary between the two is gone.  The last
// dense block (ticket on sync[1]) resets both words for the next launch.  Only for grids of <= 256 blocks:
// one block per CU keeps every block resident, so no poller waits on an undispatched producer; every
// spin is bounded anyway (sync[2] = 1 records a timeout).
template <int MM, int U>
__global__ __launch_bounds__(512) void attn_dense_kernel(AttnArgs a, AttnParts pa, const bf16* __restrict__ W, int M,
                                                         int N, int K, Epi ep, int nsplit, int n_attn, int n_dense,
                                                         unsigned* sync) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = blockIdx.x;
  if (bid < n_attn) {
    const int head = bid % a.n_head, rest = bid / a.n_head;
    attn_decode_block<bf16, 8, 32, true>(a, head, rest % a.B, rest / a.B, nsplit, sync);
    return;
  }
  gemv_rows_block<1, MM, U, X_PARTS, 0, true>(W, nullptr, LnArgs{}, pa, M, N, K, ep, bid - n_attn, smem, sync,
                                     (unsigned)n_attn);
  if (threadIdx.x == 0) {  // this lane's poll matched above: the last dense block resets the words
    typedef __attribute__((address_space(1))) unsigned gu32;
    const unsigned old = __hip_atomic_fetch_add((gu32*)(sync + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)n_dense - 1) {
      __hip_atomic_store((gu32*)sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32*)(sync + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static bool attn_dense_supported(int M, int N, int K, int n_head, int head_dim, int nsplit) {
  const int n_attn = M * n_head * nsplit, n_dense = (N + 7) / 8;
  return M >= 1 && M <= 2 && nsplit >= 2 && nsplit <= kPartsMaxSplit && head_dim <= 128 && head_dim % 8 == 0 &&
         K % 512 == 0 && K <= 4096 && K == n_head * head_dim && n_attn + n_dense <= 256;
}

static void launch_attn_dense(const AttnArgs& a, const void* W, int M, int N, int K, const Epi& ep, unsigned* sync,
                       hipStream_t s) {
  const int nsplit = attention_decode_splits(a.B, a.n_head, a.max_chunks);
  const AttnParts pa{a.part_acc, a.part_ml, nsplit, a.n_head, a.head_dim, a.max_chunks, a.slot};
  const int n_attn = M * a.n_head * nsplit, n_dense = (N + 7) / 8;
  const size_t shm = 256 + (size_t)M * K * sizeof(bf16);
  // U: 512-column chunks per row in flight, the rows_plan choice for 8-wave R = 1 blocks (<= 8 registers' worth)
  const int cpr = K / 512;
  const int u = cpr <= 3 || cpr == 5 || cpr == 8 ? cpr : (cpr % 4 == 0 ? 4 : (cpr % 2 == 0 ? 2 : 1));
  auto go = [&](auto mc, auto uc) {
    constexpr int MMc = decltype(mc)::value, Uc = decltype(uc)::value;
    attn_dense_kernel<MMc, Uc><<<n_attn + n_dense, 512, shm, s>>>(a, pa, (const bf16*)W, M, N, K, ep, nsplit,
                                                                  n_attn, n_dense, sync);
  };
  auto gm = [&](auto uc) {
    if (M == 1) go(EpiKindC<1>{}, uc);
    else go(EpiKindC<2>{}, uc);
  };
  switch (u) {
    case 1: gm(EpiKindC<1>{}); break;
    case 2: gm(EpiKindC<2>{}); break;
    case 3: gm(EpiKindC<3>{}); break;
    case 5: gm(EpiKindC<5>{}); break;
    case 8: gm(EpiKindC<8>{}); break;
    default: gm(EpiKindC<4>{}); break;
  }
}


#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const int nh = 16, hd = 96, h = nh * hd, max_ctx = 700, B = 1, past = 600;
  int max_chunks, chunk;
  const size_t wsf = attention_workspace_floats(B, nh, hd, max_ctx, &max_chunks, &chunk);
  const size_t kv = (size_t)B * nh * max_ctx * hd;
  bf16 *kc, *vc, *q, *W, *bias;
  float *resid, *out0, *out1, *ws, *slopes;
  unsigned *tickets, *sync;
  CK(hipMalloc(&kc, kv * 2)); CK(hipMalloc(&vc, kv * 2)); CK(hipMalloc(&q, h * 2)); CK(hipMalloc(&W, (size_t)h * h * 2));
  CK(hipMalloc(&bias, h * 2)); CK(hipMalloc(&resid, h * 4)); CK(hipMalloc(&out0, h * 4)); CK(hipMalloc(&out1, h * 4));
  CK(hipMalloc(&ws, wsf * 4 * 2)); CK(hipMalloc(&slopes, nh * 4)); CK(hipMalloc(&tickets, 4096)); CK(hipMalloc(&sync, 64));
  CK(hipMemset(tickets, 0, 4096)); CK(hipMemset(sync, 0, 64));
  launch_gen_fill(kc, 1, kv, 11, 0, 0); launch_gen_fill(vc, 1, kv, 12, 0, 0); launch_gen_fill(q, 1, h, 13, 0, 0);
  launch_gen_fill(W, 1, (size_t)h * h, 14, 0, 0); launch_gen_fill(bias, 1, h, 15, 1, 0);
  launch_gen_fill(resid, 0, h, 16, 0, 0);
  std::vector<float> sl(nh);
  for (int i = 0; i < nh; i++) sl[i] = powf(2.f, -8.f * (i + 1) / nh);  // n_head a power of two (ALiBi)
  CK(hipMemcpy(slopes, sl.data(), nh * 4, hipMemcpyHostToDevice));
  AttnArgs a{};
  a.q = q; a.k_cache = kc; a.v_cache = vc; a.ctx_out = nullptr; a.slopes = slopes; a.B = B; a.S = 1; a.slot = 0;
  a.past = past; a.n_head = nh; a.head_dim = hd; a.max_ctx = max_ctx; a.hidden = h; a.inv_norm = 1.0f / sqrtf((float)hd);
  a.part_acc = ws; a.part_ml = ws + (size_t)B * nh * max_chunks * hd; a.max_chunks = max_chunks; a.chunk = chunk;
  a.tickets = tickets; a.defer_merge = 1;
  const int nsplit = attention_decode_splits(B, nh, max_chunks);
  if (!attn_dense_supported(B, h, h, nh, hd, nsplit) || !linear_parts_supported(B, h, hd, nsplit)) { printf("unsupported\n"); return 1; }
  const AttnParts parts{a.part_acc, a.part_ml, nsplit, nh, hd, max_chunks, 0};
  Epi e{};
  e.kind = EPI_RESID; e.bias = bias; e.resid = resid; e.ldo = h;
  auto separate = [&](float* o) { e.out_f32 = o; launch_attention(1, a, 0); launch_linear_parts(parts, W, B, h, h, e, 0); };
  auto fused = [&](float* o) { e.out_f32 = o; launch_attn_dense(a, W, B, h, h, e, sync, 0); };
  separate(out0); fused(out1);
  CK(hipDeviceSynchronize());
  std::vector<float> h0(h), h1(h);
  CK(hipMemcpy(h0.data(), out0, h * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(h1.data(), out1, h * 4, hipMemcpyDeviceToHost));
  unsigned flag[3];
  CK(hipMemcpy(flag, sync, 12, hipMemcpyDeviceToHost));
  int diff = 0;
  for (int i = 0; i < h; i++) diff += h0[i] != h1[i];
  printf("bloom-1b1 B=1 ctx %d, %d splits: fused vs separate outputs differing: %d of %d; sync words %u %u %u\n", past + 1,
         nsplit, diff, h, flag[0], flag[1], flag[2]);
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  for (int arm = 0; arm < 4; arm++) {
    const bool f = arm & 1;
    CK(hipEventRecord(t0, 0));
    for (int i = 0; i < 200; i++) f ? fused(out1) : separate(out0);
    CK(hipEventRecord(t1, 0));
    CK(hipEventSynchronize(t1));
    float ms;
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("%-9s %7.2f us per (attention, dense) pair\n", f ? "fused" : "separate", ms * 1e3f / 200);
  }
  return diff ? 2 : 0;
}
