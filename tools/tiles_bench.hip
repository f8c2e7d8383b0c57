// tools/tiles_bench.hip — batched decode GEMV geometry sweep (round 5).  For each BLOOM block matrix and
// M = 2 / 4 / 8 / 16 / 32 rows: the library's path (launch_linear_ln / launch_linear: what a decode step runs) and gemv_ldsw4 at every
// (T tiles per block, KS K splits, waves) whose K parts divide K.  The weights rotate over copies totalling > 512 MB so
// every launch streams from HBM (not the 256 MB Infinity Cache), as in a decode step.  Time = median over 5 groups of
// (copies) back-to-back launches between HIP events.  Per-CU bytes: the busiest CU's weight + activation bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/tiles_bench.hip
//        distributed_inference_demo_amd/csrc/attn_prefill.hip -o tools/tiles_bench
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Arm { std::string name; float us; };

int main(int argc, char** argv) {
  struct Sh { const char* name; int N, K; bool ln; } shapes[] = {
      {"1b1 qkv", 4608, 1536, true}, {"1b1 dense", 1536, 1536, false}, {"1b1 fc1", 6144, 1536, true},
      {"1b1 fc2", 1536, 6144, false}, {"560m qkv", 3072, 1024, true}, {"560m dense", 1024, 1024, false},
      {"560m fc1", 4096, 1024, true}, {"560m fc2", 1024, 4096, false}, {"7b1 qkv", 12288, 4096, true},
      {"7b1 fc1", 16384, 4096, true}, {"7b1 dense", 4096, 4096, false}, {"7b1 fc2", 4096, 16384, false},
      {"3b qkv", 7680, 2560, true}, {"3b dense", 2560, 2560, false}, {"3b fc1", 10240, 2560, true},
      {"3b fc2", 2560, 10240, false}};
  const size_t pool_bytes = (size_t)640 << 20;
  char* pool;
  CK(hipMalloc(&pool, pool_bytes));
  launch_gen_fill(pool, 1, pool_bytes / 2, 7, 0, 0);
  bf16 *X, *gamma, *beta, *bias, *xn, *out;
  float *x32, *ws;
  unsigned* tick;
  CK(hipMalloc(&X, 32 * 16384 * 2)); CK(hipMalloc(&x32, 32 * 16384 * 4)); CK(hipMalloc(&xn, 32 * 16384 * 2));
  CK(hipMalloc(&gamma, 16384 * 2)); CK(hipMalloc(&beta, 16384 * 2)); CK(hipMalloc(&bias, 16384 * 2));
  CK(hipMalloc(&out, 32 * 16384 * 2));
  const size_t cap = (size_t)4 << 20;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  launch_gen_fill(X, 1, 32 * 16384, 8, 0, 0); launch_gen_fill(x32, 0, 32 * 16384, 9, 0, 0);
  launch_gen_fill(gamma, 1, 16384, 10, 2, 0); launch_gen_fill(beta, 1, 16384, 11, 1, 0);
  launch_gen_fill(bias, 1, 16384, 12, 1, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* only = argc > 1 && strcmp(argv[1], "all") ? argv[1] : nullptr;  // tiles_bench [shape filter|all] [M]
  const int mlist[5] = {2, 4, 8, 16, 32};
  for (int M : mlist) {
    if (argc > 2 && M != atoi(argv[2])) continue;
    for (auto& sh : shapes) {
      if (only && !strstr(sh.name, only)) continue;
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
      std::vector<Arm> arms;
      const float lib = time([&](const bf16* W) {
        if (sh.ln) launch_linear_ln(1, x32, 1, 0, gamma, beta, 1e-5f, xn, W, M, sh.N, sh.K, ep, 0);
        else launch_linear(1, X, W, M, sh.N, sh.K, ep, 0);
      });
      const float lnk = sh.ln ? time([&](const bf16*) {
        launch_ln_rows(x32, 1, 0, gamma, beta, 1e-5f, xn, M, sh.K, 0);
      }) : 0.f;
      const float plain = time([&](const bf16* W) { launch_linear(1, X, W, M, sh.N, sh.K, ep, 0); });
      auto arm = [&](auto tc, auto wc, auto mc, int KS) {
        constexpr int T = decltype(tc)::value, WV = decltype(wc)::value, MT = decltype(mc)::value;
        const int blocks = (sh.N + T * 16 - 1) / (T * 16);
        if (sh.K % (KS * WV * 64) || blocks > 4096 || (KS > 1 && (size_t)KS * M * sh.N > cap)) return;
        const float us = time([&](const bf16* W) { gemv_ldsw4_launch<T, WV, MT, bf16>(X, W, M, sh.N, sh.K, KS, ep, 0); });
        char nm[64];
        snprintf(nm, sizeof nm, "T%d KS%d W%d (%d blk)", T, KS, WV, blocks * KS);
        arms.push_back({nm, us});
      };
      for (int KS : {1, 2, 3, 4, 6, 8}) {
        auto per_t = [&](auto wc) {
          if (M <= 16) {
            arm(EpiKindC<1>{}, wc, EpiKindC<1>{}, KS); arm(EpiKindC<2>{}, wc, EpiKindC<1>{}, KS);
            arm(EpiKindC<3>{}, wc, EpiKindC<1>{}, KS); arm(EpiKindC<4>{}, wc, EpiKindC<1>{}, KS);
          } else {
            arm(EpiKindC<1>{}, wc, EpiKindC<2>{}, KS); arm(EpiKindC<2>{}, wc, EpiKindC<2>{}, KS);
            arm(EpiKindC<3>{}, wc, EpiKindC<2>{}, KS); arm(EpiKindC<4>{}, wc, EpiKindC<2>{}, KS);
          }
        };
        per_t(EpiKindC<4>{});
        per_t(EpiKindC<8>{});
      }
      std::sort(arms.begin(), arms.end(), [](const Arm& a, const Arm& b) { return a.us < b.us; });
      printf("M=%2d %-10s N=%5d K=%5d  library %6.2f us%s", M, sh.name, sh.N, sh.K, lib, sh.ln ? " (LN)" : "");
      if (sh.ln) printf("  [LN launch %5.2f + plain GEMV %6.2f]", lnk, plain);
      printf("  %5.0f GB/s\n", wb / (lib * 1e-6) / 1e9);
      for (size_t i = 0; i < arms.size() && i < 6; i++)
        printf("      %-22s %6.2f us  %5.0f GB/s\n", arms[i].name.c_str(), arms[i].us, wb / (arms[i].us * 1e-6) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
