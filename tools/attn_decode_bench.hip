// tools/attn_decode_bench.hip — single-split decode attention (attn_decode_kernel, S = 1) with 8-wave blocks
// (one per CU at 228 VGPRs) against 4-wave blocks (two per CU) on batched-decode shapes; HIP events, median of
// 20 launches; the 4-wave output is compared with the 8-wave one (max |diff| of the bf16 context).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/attn_decode_bench.hip -o tools/attn_decode_bench
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
  struct Sh { const char* name; int B, nh, hd, ctx; } shapes[] = {
      {"1b1 B=32", 32, 16, 96, 164}, {"1b1 B=32", 32, 16, 96, 580}, {"1b1 B=8", 8, 16, 96, 164},
      {"7b1 B=32", 32, 32, 128, 164}, {"7b1 B=32", 32, 32, 128, 1044}, {"7b1 B=32", 32, 32, 128, 2004},
      {"560m B=32", 32, 16, 64, 84}};
  const int max_ctx = 2048;
  const size_t kvn = (size_t)32 * 32 * max_ctx * 128;
  bf16 *q, *kc, *vc, *ctx; float* slopes; int* pastd;
  CK(hipMalloc(&q, (size_t)32 * 4096 * 2)); CK(hipMalloc(&ctx, (size_t)32 * 4096 * 2));
  CK(hipMalloc(&kc, kvn * 2)); CK(hipMalloc(&vc, kvn * 2));
  CK(hipMalloc(&slopes, 64 * 4)); CK(hipMalloc(&pastd, 64 * 4));
  fill_rand<<<4096, 256>>>(q, (size_t)32 * 4096, 1, 2.f); fill_rand<<<4096, 256>>>(kc, kvn, 2, 2.f); fill_rand<<<4096, 256>>>(vc, kvn, 3, 2.f);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    std::vector<float> hs(64);
    for (int i = 0; i < sh.nh; i++) hs[i] = powf(2.f, -8.f * (i + 1) / sh.nh);
    CK(hipMemcpy(slopes, hs.data(), 64 * 4, hipMemcpyHostToDevice));
    std::vector<int> hp(64, sh.ctx - 1);
    CK(hipMemcpy(pastd, hp.data(), 64 * 4, hipMemcpyHostToDevice));
    AttnArgs a{};
    a.q = q; a.k_cache = kc; a.v_cache = vc; a.ctx_out = ctx; a.slopes = slopes;
    a.B = sh.B; a.S = 1; a.slot = 0; a.past_dev = pastd; a.past = sh.ctx - 1; a.n_head = sh.nh; a.head_dim = sh.hd;
    a.max_ctx = max_ctx; a.hidden = sh.nh * sh.hd; a.inv_norm = 1.f / sqrtf((float)sh.hd); a.chunk = 64;
    const size_t on = (size_t)sh.B * a.hidden;
    std::vector<bf16> h8(on), h4(on);
    const dim3 g(sh.nh, sh.B, 1);
    auto timeit = [&](auto&& fn) {
      std::vector<float> t;
      for (int it = 0; it < 25; it++) {
        CK(hipEventRecord(e0)); fn(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      return t[t.size() / 2];
    };
    const float t8 = timeit([&] { attn_decode_kernel<bf16, 8><<<g, 512>>>(a); });
    CK(hipMemcpy(h8.data(), ctx, on * 2, hipMemcpyDeviceToHost));
    const float t4 = timeit([&] { attn_decode_kernel<bf16, 4><<<g, 256>>>(a); });
    CK(hipMemcpy(h4.data(), ctx, on * 2, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < on; i++) md = std::max(md, (double)fabsf((float)h4[i] - (float)h8[i]));
    const double kv = 2.0 * sh.B * sh.nh * (double)sh.ctx * sh.hd * 2;
    printf("%-10s pairs %4d ctx %4d hd %3d  8 waves %7.2f us (%5.2f TB/s)  4 waves %7.2f us (%5.2f TB/s)  max|diff| %.3g\n",
           sh.name, sh.B * sh.nh, sh.ctx, sh.hd, t8, kv / t8 * 1e-6, t4, kv / t4 * 1e-6, md);
  }
  return 0;
}
