// tools/rows_m_probe.hip — how the rows GEMV (gemv_rows_kernel: dot products on v_dot2, weights streamed once per
// wave, every token's activation row read per chunk) scales with the token count M, against the library's batched
// path (launch_linear at M = 8: gemv_ldsw4, MFMA tiles).  Plain GEMVs (no LayerNorm prologue), bloom-1b1 / 3b block
// matrices, weights rotated over > 512 MB (HBM-cold).  Median of 5 groups of back-to-back launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/rows_m_probe.hip
//        distributed_inference_demo_amd/csrc/attn_prefill.hip -o tools/rows_m_probe
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  struct Sh { const char* name; int N, K; } shapes[] = {
      {"1b1 qkv", 4608, 1536}, {"1b1 dense", 1536, 1536}, {"1b1 fc1", 6144, 1536}, {"1b1 fc2", 1536, 6144},
      {"3b qkv", 7680, 2560}, {"3b dense", 2560, 2560}, {"3b fc1", 10240, 2560}, {"3b fc2", 2560, 10240}};
  const size_t pool_bytes = (size_t)640 << 20;
  char* pool;
  CK(hipMalloc(&pool, pool_bytes));
  launch_gen_fill(pool, 1, pool_bytes / 2, 7, 0, 0);
  bf16 *X, *bias, *out;
  float *ws;
  unsigned* tick;
  CK(hipMalloc(&X, 16 * 16384 * 2)); CK(hipMalloc(&bias, 16384 * 2)); CK(hipMalloc(&out, 16 * 16384 * 2));
  const size_t cap = (size_t)4 << 20;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  launch_gen_fill(X, 1, 16 * 16384, 8, 0, 0); launch_gen_fill(bias, 1, 16384, 12, 1, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    const size_t wb = (size_t)sh.N * sh.K * 2;
    const int ncopy = (int)std::min<size_t>(64, pool_bytes / wb);
    Epi ep{};
    ep.kind = EPI_GELU; ep.bias = bias; ep.ldo = sh.N; ep.out_act = out;
    ep.sk_ws = ws; ep.sk_tickets = tick; ep.sk_cap = cap; ep.sk_ntickets = 4096;
    auto time = [&](const std::function<void(const bf16*)>& f) {
      std::vector<float> t;
      for (int c = 0; c < ncopy; c++) f((const bf16*)(pool + (size_t)c * wb));
      CK(hipDeviceSynchronize());
      for (int g = 0; g < 5; g++) {
        CK(hipEventRecord(e0));
        for (int c = 0; c < ncopy; c++) f((const bf16*)(pool + (size_t)c * wb));
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3f / ncopy);
      }
      std::sort(t.begin(), t.end());
      return t[2];
    };
    int R, waves, U;
    float rows[3];
    const int ms[3] = {1, 2, 4};
    for (int i = 0; i < 3; i++) {
      const int M = ms[i];
      rows_plan(X_PLAIN, M, sh.N, sh.K, &R, &waves, &U);
      rows[i] = time([&](const bf16* W) {
        if (M == 1) gemv_rows_launch<2, 1, X_PLAIN, 4>(X, LnArgs{}, AttnParts{}, W, M, sh.N, sh.K, ep, 0, 4);
        else if (M == 2) gemv_rows_launch<2, 2, X_PLAIN, 4>(X, LnArgs{}, AttnParts{}, W, M, sh.N, sh.K, ep, 0, 4);
        else gemv_rows_launch<2, 4, X_PLAIN, 4>(X, LnArgs{}, AttnParts{}, W, M, sh.N, sh.K, ep, 0, 4);
      });
    }
    const float lib1 = time([&](const bf16* W) { launch_linear(1, X, W, 1, sh.N, sh.K, ep, 0); });
    const float lib4 = time([&](const bf16* W) { launch_linear(1, X, W, 4, sh.N, sh.K, ep, 0); });
    const float lib8 = time([&](const bf16* W) { launch_linear(1, X, W, 8, sh.N, sh.K, ep, 0); });
    const float lib16 = time([&](const bf16* W) { launch_linear(1, X, W, 16, sh.N, sh.K, ep, 0); });
    printf("%-10s N=%5d K=%5d  rows R2 U4 4-wave blocks: M=1 %6.2f  M=2 %6.2f  M=4 %6.2f us | library M=1 %6.2f  "
           "M=4 %6.2f  M=8 %6.2f  M=16 %6.2f us\n",
           sh.name, sh.N, sh.K, rows[0], rows[1], rows[2], lib1, lib4, lib8, lib16);
    fflush(stdout);
  }
  return 0;
}
