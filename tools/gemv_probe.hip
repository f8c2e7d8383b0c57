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
