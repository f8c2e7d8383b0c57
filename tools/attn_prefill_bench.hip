// tools/attn_prefill_bench.hip — prefill attention (attn_prefill_mfma_kernel) timing on the BLOOM prefill shapes,
// HIP events, median of 20 launches: no split (pf_tiles = 0) against split-KV with 1 / 2 / 4 key tiles per
// block; every split output is compared with the unsplit one (max |diff| of the bf16 context printed).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/attn_prefill_bench.hip -o tools/attn_prefill_bench
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
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

int main() {
  struct Sh { const char* name; int B, S, past, nh, hd; } shapes[] = {
      {"1b1 S512", 1, 512, 0, 16, 96}, {"560m S512", 1, 512, 0, 16, 64}, {"3b S512", 1, 512, 0, 32, 80},
      {"7b1 S512", 1, 512, 0, 32, 128}, {"1b1 S128", 1, 128, 0, 16, 96}, {"1b1 S256+past768", 1, 256, 768, 16, 96}};
  const int max_ctx = 2048;
  bf16 *q, *kc, *vc, *ctx, *ref; float *slopes, *ws; unsigned* tick; int* pastd;
  const size_t qn = (size_t)2 * 1024 * 4096;
  const size_t kvn = (size_t)2 * 32 * max_ctx * 128;
  CK(hipMalloc(&q, qn * 2)); CK(hipMalloc(&ctx, qn * 2)); CK(hipMalloc(&ref, qn * 2));
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
    a.pf_ws = ws; a.pf_cap = cap; a.pf_tickets = tick; a.pf_ntickets = 4096; a.pf_past_max = sh.past;
    const size_t on = (size_t)sh.B * sh.S * a.hidden;
    std::vector<bf16> hr(on), ho(on);
    for (int pt : {0, 1, 2, 4}) {
      a.pf_tiles = pt;
      std::vector<float> t;
      for (int it = 0; it < 25; it++) {
        CK(hipEventRecord(e0)); launch_attention(1, a, 0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      double md = 0;
      if (pt == 0) {
        CK(hipMemcpy(hr.data(), ctx, on * 2, hipMemcpyDeviceToHost));
      } else {
        CK(hipMemcpy(ho.data(), ctx, on * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < on; i++) md = std::max(md, (double)fabsf((float)ho[i] - (float)hr[i]));
      }
      printf("%-18s B=%d S=%4d past=%4d nh=%2d hd=%3d  pf_tiles=%d  median %7.2f us  min %7.2f  max|diff| %.3g\n", sh.name,
             sh.B, sh.S, sh.past, sh.nh, sh.hd, pt, t[t.size() / 2], t[0], md);
    }
    // 32-query blocks (2 waves): twice the blocks, each staging a key tile for half the queries
    for (int pt : {0, 2, 4}) {
      a.pf_tiles = pt;
      std::vector<float> t;
      for (int it = 0; it < 25; it++) {
        CK(hipEventRecord(e0)); attn_prefill_mfma_launch<2>(a, 0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      CK(hipMemcpy(ho.data(), ctx, on * 2, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < on; i++) md = std::max(md, (double)fabsf((float)ho[i] - (float)hr[i]));
      printf("%-18s B=%d S=%4d past=%4d nh=%2d hd=%3d  QW=2 pf_tiles=%d  median %7.2f us  min %7.2f  max|diff| %.3g\n",
             sh.name, sh.B, sh.S, sh.past, sh.nh, sh.hd, pt, t[t.size() / 2], t[0], md);
    }
  }
  return 0;
}
