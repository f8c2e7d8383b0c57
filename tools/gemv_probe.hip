// tools/gemv_probe.hip — where does a decode GEMV lose time against a pure stream of the same bytes?
// Times gemv_rows_kernel with probe flags (FL: 1 = temporal weight loads, 2 = no activation
// loads, 4 = no epilogue), LN vs plain prologue, rows per wave, plus stream reads and an empty
// launch of the same grid.  Cold weights (a 2 GB rotation).  M = 1, bloom-1b1 shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemv_probe.hip -o tools/gemv_probe
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = d_lb32((uint32_t)i ^ seed);
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * 0.04f);
  }
}
__global__ void fill_f(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (float)((i * 2654435761u) % 1000) / 500.0f - 1.0f;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int NT>
__global__ __launch_bounds__(256) void stream_read(const u32x4* p, size_t n, u32x4* sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= NT ? __builtin_nontemporal_load(p + i) : p[i];
  if (acc.x == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void empty_kernel(int* sink) {
  if (threadIdx.x == 1023) sink[0] = 1;
}

int main() {
  struct Shape { const char* name; int N, K; bool ln; int R, U; } shapes[] = {
    {"1b1 qkv", 4608, 1536, true, 1, 3}, {"1b1 dense", 1536, 1536, false, 1, 3},
    {"1b1 fc1", 6144, 1536, true, 2, 3}, {"1b1 fc2", 1536, 6144, false, 1, 12},
  };
  const size_t maxW = (size_t)1 << 30;  // 1 G elements = 2 GB rotation
  bf16 *W, *X, *gb, *act; float *xf, *outf; unsigned long long* keys; u32x4* sink;
  CK(hipMalloc(&W, maxW * 2)); CK(hipMalloc(&X, 16384 * 2)); CK(hipMalloc(&xf, 16384 * 4));
  CK(hipMalloc(&outf, 32768 * 4)); CK(hipMalloc(&gb, 16384 * 2 * 2)); CK(hipMalloc(&act, 32768 * 2));
  CK(hipMalloc(&keys, 4096 * 8)); CK(hipMalloc(&sink, 64));
  fill_rand<<<4096, 256>>>(W, maxW, 1); fill_rand<<<64, 256>>>(X, 16384, 2); fill_f<<<64, 256>>>(xf, 16384);
  fill_rand<<<64, 256>>>(gb, 2 * 16384, 3);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int REPS = 50, ROUNDS = 5;
  // launch floor: empty kernels of several grid sizes, stream launches vs one captured graph
  if (getenv("PROBE_LAUNCH")) {
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int g : {1, 64, 256, 1024, 4096}) {
      float best_s = 1e9f, best_g = 1e9f;
      hipGraph_t gr; hipGraphExec_t ex;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < REPS; i++) empty_kernel<<<g, 256, 0, st>>>((int*)sink);
      CK(hipStreamEndCapture(st, &gr)); CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
      for (int r = 0; r < ROUNDS; r++) {
        float ms;
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < REPS; i++) empty_kernel<<<g, 256, 0, st>>>((int*)sink);
        CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        best_s = std::min(best_s, ms * 1e3f / REPS);
        CK(hipGraphLaunch(ex, st));
        CK(hipEventRecord(e0, st)); CK(hipGraphLaunch(ex, st));
        CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        best_g = std::min(best_g, ms * 1e3f / REPS);
      }
      printf("empty kernel grid %5d x 256: stream %.2f us/launch, graph %.2f us/launch\n", g, best_s, best_g);
    }
    return 0;
  }
  // sweep of the tile GEMV's (T, KS, waves) per batched shape: best configurations first
  if (getenv("PROBE_SWEEP")) {
    struct BS { const char* name; int N, K; } bsh[] = {
      {"1b1 qkv", 4608, 1536}, {"1b1 dense", 1536, 1536}, {"1b1 fc1", 6144, 1536}, {"1b1 fc2", 1536, 6144},
      {"3b qkv", 7680, 2560}, {"3b dense", 2560, 2560}, {"3b fc1", 10240, 2560}, {"3b fc2", 2560, 10240},
      {"7b1 qkv", 12288, 4096}, {"7b1 dense", 4096, 4096}, {"7b1 fc1", 16384, 4096}, {"7b1 fc2", 4096, 16384}};
    bf16* xn; CK(hipMalloc(&xn, 32 * 16384 * 2)); fill_rand<<<64, 256>>>(xn, 32 * 16384, 5);
    float* bout; CK(hipMalloc(&bout, (size_t)32 * 16384 * 4));
    float* skws; unsigned* sktk;
    const size_t cap = (size_t)16 * 32 * 4096;
    CK(hipMalloc(&skws, cap * 4)); CK(hipMalloc(&sktk, 4096 * 4)); CK(hipMemset(sktk, 0, 4096 * 4));
    CK(hipDeviceSynchronize());
    for (int M : {8, 32}) {
      for (auto& sh : bsh) {
        const int N = sh.N, K = sh.K, units = K / 64;
        Epi ep{};
        ep.kind = EPI_RESID; ep.bias = gb; ep.out_f32 = bout; ep.resid = bout; ep.ldo = N;
        ep.sk_ws = skws; ep.sk_tickets = sktk; ep.sk_cap = cap; ep.sk_ntickets = 4096;
        const size_t nk = (size_t)N * K, rot = (maxW - nk) / 256 + 1;
        std::vector<std::pair<float, std::string>> res;
        for (int T : {1, 2, 4})
          for (int KS : {1, 2, 4, 8})
            for (int WV : {4, 8, 16}) {
              if (WV == 16 && T != 1) continue;
              if ((size_t)KS * M * N > cap || units / KS < WV || (N / (16 * T)) > 4096) continue;
              auto f = [&](const bf16* w) {
                const bool two = M > 16;
#define TL(TT, WW) do { if (two) gemv_tiles_launch<TT, 2, WW>(xn, w, M, N, K, KS, ep, 0); else gemv_tiles_launch<TT, 1, WW>(xn, w, M, N, K, KS, ep, 0); } while (0)
                if (T == 1) { if (WV == 4) TL(1, 4); else if (WV == 8) TL(1, 8); else TL(1, 16); }
                else if (T == 2) { if (WV == 4) TL(2, 4); else TL(2, 8); }
                else { if (WV == 4) TL(4, 4); else TL(4, 8); }
#undef TL
              };
              std::vector<float> t;
              for (int r = 0; r < 3; r++) {
                f(W);
                CK(hipEventRecord(e0));
                for (int i = 0; i < 20; i++) f(W + (((size_t)(i + r * 20) * (nk / 256 + 7)) % rot) * 256);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t.push_back(ms * 1e3f / 20);
              }
              std::sort(t.begin(), t.end());
              char buf[64]; snprintf(buf, sizeof buf, "T=%d KS=%d WV=%d", T, KS, WV);
              res.push_back({t[1], buf});
            }
        std::sort(res.begin(), res.end());
        const int mine_T = (N + 63) / 64 >= 256 ? 4 : ((N + 31) / 32 >= 256 ? 2 : 1);
        printf("M=%2d %-10s N=%6d K=%5d %.1f MB:", M, sh.name, N, K, nk * 2 / 1e6);
        for (size_t i = 0; i < res.size() && i < 4; i++) printf("  %s %.2fus", res[i].second.c_str(), res[i].first);
        printf("  | worst %s %.2fus\n", res.back().second.c_str(), res.back().first);
        (void)mine_T;
      }
    }
    CK(hipGetLastError());
    return 0;
  }
  // batched decode: the per-tile MFMA GEMV (old) vs the tile GEMV (+ a LayerNorm kernel for LN shapes)
  if (getenv("PROBE_BATCH")) {
    struct BS { const char* name; int N, K; bool ln; } bsh[] = {
      {"1b1 qkv", 4608, 1536, true}, {"1b1 dense", 1536, 1536, false}, {"1b1 fc1", 6144, 1536, true},
      {"1b1 fc2", 1536, 6144, false}, {"1b1 lm_head", 250880, 1536, true},
      {"7b1 qkv", 12288, 4096, true}, {"7b1 dense", 4096, 4096, false}, {"7b1 fc1", 16384, 4096, true},
      {"7b1 fc2", 4096, 16384, false}};
    bf16* xn; float* xf32; unsigned long long* bkeys;
    CK(hipMalloc(&xn, 32 * 16384 * 2)); CK(hipMalloc(&xf32, 32 * 16384 * 4)); CK(hipMalloc(&bkeys, 32 * 15680 * 8));
    float* bout; CK(hipMalloc(&bout, (size_t)32 * 16384 * 4));
    float* skws; unsigned* sktk;
    CK(hipMalloc(&skws, (size_t)16 * 32 * 4096 * 4)); CK(hipMalloc(&sktk, 4096 * 4)); CK(hipMemset(sktk, 0, 4096 * 4));
    fill_f<<<64, 256>>>(xf32, 32 * 16384); fill_rand<<<64, 256>>>(xn, 32 * 16384, 5);
    CK(hipDeviceSynchronize());
    for (int M : {8, 32}) {
      for (auto& sh : bsh) {
        const int N = sh.N, K = sh.K;
        Epi ep{};
        if (N == 250880) { ep.kind = EPI_ARGMAX; ep.keys = bkeys; ep.ldo = N; }
        else { ep.kind = EPI_RESID; ep.bias = gb; ep.out_f32 = bout; ep.resid = bout; ep.ldo = N; }
        Epi eps = ep;
        eps.sk_ws = skws; eps.sk_tickets = sktk; eps.sk_cap = (size_t)16 * 32 * 4096; eps.sk_ntickets = 4096;
        LnArgs ln{xf32, 1, 0, gb, gb + 16384, 1e-5f};
        const size_t nk = (size_t)N * K, units = nk > maxW ? 1 : (maxW - nk) / 256 + 1;
        typedef std::function<void(const bf16*)> F;
        std::vector<std::pair<std::string, F>> vars;
        const int waves = gemv_waves(N, K);
        vars.push_back({"old mfma", [&](const bf16* w) {
          const bool two = M > 16;
          if (sh.ln && M <= 8) {
            if (waves == 4) gemv_launch<4, 1, true>(nullptr, ln, w, M, N, K, ep, 0);
            else if (waves == 8) gemv_launch<8, 1, true>(nullptr, ln, w, M, N, K, ep, 0);
            else gemv_launch<16, 1, true>(nullptr, ln, w, M, N, K, ep, 0);
          } else {
            if (sh.ln) launch_layernorm(1, xf32, nullptr, 1, 0, gb, gb + 16384, xn, 0, M, K, 1e-5f, 0);
            if (waves == 4) { if (two) gemv_launch<4, 2, false>(xn, ln, w, M, N, K, ep, 0); else gemv_launch<4, 1, false>(xn, ln, w, M, N, K, ep, 0); }
            else if (waves == 8) { if (two) gemv_launch<8, 2, false>(xn, ln, w, M, N, K, ep, 0); else gemv_launch<8, 1, false>(xn, ln, w, M, N, K, ep, 0); }
            else { if (two) gemv_launch<16, 2, false>(xn, ln, w, M, N, K, ep, 0); else gemv_launch<16, 1, false>(xn, ln, w, M, N, K, ep, 0); }
          }
        }});
        vars.push_back({"tiles (+ln_rows)", [&](const bf16* w) {
          if (sh.ln) launch_ln_rows_wave(ln, M, K, xn, 0);
          gemv_tiles_dispatch(xn, w, M, N, K, eps, 0);
        }});
        if (sh.ln) vars.push_back({"tiles (no LN)", [&](const bf16* w) { gemv_tiles_dispatch(xn, w, M, N, K, eps, 0); }});
        else vars.push_back({"tiles (no split-K)", [&](const bf16* w) { gemv_tiles_dispatch(xn, w, M, N, K, ep, 0); }});
        vars.push_back({"stream nt", [&](const bf16* w) { stream_read<1><<<2048, 256>>>((const u32x4*)w, nk * 2 / 16, sink); }});
        std::vector<std::vector<float>> t(vars.size());
        for (int r = 0; r < ROUNDS; r++)
          for (size_t v = 0; v < vars.size(); v++) {
            for (int i = 0; i < 2; i++) vars[v].second(W);
            CK(hipEventRecord(e0));
            for (int i = 0; i < 20; i++) vars[v].second(W + (((size_t)(i + r * 20) * (nk / 256 + 7)) % units) * 256);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1e3f / 20);
          }
        printf("M=%2d %-12s N=%6d K=%5d  %.1f MB\n", M, sh.name, N, K, nk * 2 / 1e6);
        for (size_t v = 0; v < vars.size(); v++) {
          std::sort(t[v].begin(), t[v].end());
          printf("   %-20s median %8.2f us  %6.0f GB/s\n", vars[v].first.c_str(), t[v][ROUNDS / 2],
                 nk * 2 / (t[v][ROUNDS / 2] * 1e-6) / 1e9);
        }
      }
    }
    CK(hipGetLastError());
    return 0;
  }
  for (auto& sh : shapes) {
    Epi ep{};
    if (sh.ln) { ep.kind = EPI_GELU; ep.bias = gb; ep.out_act = act; ep.ldo = sh.N; }
    else { ep.kind = EPI_RESID; ep.bias = gb; ep.out_f32 = outf; ep.resid = outf; ep.ldo = sh.N; }
    ep.keys = keys;
    LnArgs ln{xf, 1, 0, gb, gb + 16384, 1e-5f};
    const AttnParts pa{};
    const int M = 1, N = sh.N, K = sh.K;
    typedef std::function<void(const bf16*)> F;
    std::vector<std::pair<std::string, F>> vars;
    const int blocks = (N + 4 * sh.R - 1) / (4 * sh.R);
#define RV(NAME, R_, XM_, U_, FL_) vars.push_back({NAME, [&](const bf16* w) { gemv_rows_launch<R_, 1, XM_, U_, FL_>(X, ln, pa, w, M, N, K, ep, 0); }})
    if (sh.ln) {
      RV("prod (LN)", 1, X_LN, 3, 0);
      if (sh.R == 2) RV("prod (LN) R2", 2, X_LN, 3, 0);
      RV("LN temporal", 1, X_LN, 3, 1);
      RV("LN noepi", 1, X_LN, 3, 4);
      RV("plain (no LN)", 1, X_PLAIN, 3, 0);
      RV("plain R2", 2, X_PLAIN, 3, 0);
      RV("plain R4", 4, X_PLAIN, 3, 0);
      RV("plain temporal", 1, X_PLAIN, 3, 1);
      RV("plain nox", 1, X_PLAIN, 3, 2);
      RV("plain noepi", 1, X_PLAIN, 3, 4);
      RV("plain all-off", 1, X_PLAIN, 3, 7);
    } else if (sh.U == 3) {
      RV("prod", 1, X_PLAIN, 3, 0);
      RV("R2", 2, X_PLAIN, 3, 0);
      RV("temporal", 1, X_PLAIN, 3, 1);
      RV("nox", 1, X_PLAIN, 3, 2);
      RV("noepi", 1, X_PLAIN, 3, 4);
      RV("all-off", 1, X_PLAIN, 3, 7);
    } else {
      RV("prod", 1, X_PLAIN, 12, 0);
      RV("U6", 1, X_PLAIN, 6, 0);
      RV("U4", 1, X_PLAIN, 4, 0);
      RV("temporal", 1, X_PLAIN, 12, 1);
      RV("nox", 1, X_PLAIN, 12, 2);
      RV("noepi", 1, X_PLAIN, 12, 4);
      RV("all-off", 1, X_PLAIN, 12, 7);
    }
    const size_t bytesn = (size_t)N * K * 2 / 16;
    vars.push_back({"stream nt", [&](const bf16* w) { stream_read<1><<<2048, 256>>>((const u32x4*)w, bytesn, sink); }});
    vars.push_back({"stream plain", [&](const bf16* w) { stream_read<0><<<2048, 256>>>((const u32x4*)w, bytesn, sink); }});
    vars.push_back({"empty (same grid)", [&](const bf16*) { empty_kernel<<<blocks, 256>>>((int*)sink); }});
    std::vector<std::vector<float>> t(vars.size());
    const size_t nk = (size_t)N * K, units = (maxW - nk) / 256 + 1;
    for (int r = 0; r < ROUNDS; r++) {
      for (size_t v = 0; v < vars.size(); v++) {
        for (int i = 0; i < 3; i++) vars[v].second(W);
        CK(hipEventRecord(e0));
        for (int i = 0; i < REPS; i++) vars[v].second(W + (((size_t)(i + r * REPS) * (nk / 256 + 7)) % units) * 256);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3f / REPS);
      }
    }
    printf("%-10s N=%6d K=%5d  %.1f MB\n", sh.name, N, K, nk * 2 / 1e6);
    for (size_t v = 0; v < vars.size(); v++) {
      std::sort(t[v].begin(), t[v].end());
      printf("   %-20s median %7.2f us  min %7.2f us  %6.0f GB/s\n", vars[v].first.c_str(), t[v][ROUNDS / 2], t[v][0],
             nk * 2 / (t[v][ROUNDS / 2] * 1e-6) / 1e9);
    }
  }
  CK(hipGetLastError());
  return 0;
}
