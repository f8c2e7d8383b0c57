// tools/gemv_bench.hip — A/B microbenchmark of the decode GEMV variants (one process, interleaved
// rounds, random bf16 data).  Build: hipcc --offload-arch=gfx950 -O3 -I include tools/gemv_bench.hip
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

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
// pure streaming read of the same bytes (roofline reference)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_read(const u32x4* p, size_t n, u32x4* sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= __builtin_nontemporal_load(p + i);
  if (acc.x == 0x12345678u) sink[0] = acc;
}

typedef void (*Launch)(const bf16* W, const bf16* X, const LnArgs& ln, int M, int N, int K, const Epi& ep, hipStream_t s);

template <int WAVES, int MT, bool LN, int NT, int PF, int U>
void lv(const bf16* W, const bf16* X, const LnArgs& ln, int M, int N, int K, const Epi& ep, hipStream_t s) {
  size_t shm = sizeof(float) * WAVES * MT * 16 * 17 + (LN ? (size_t)M * K * 2 : 0);
  gemv_mfma_kernel<WAVES, MT, U, LN, NT, PF><<<(N + 15) / 16, WAVES * 64, shm, s>>>(W, X, ln, M, N, K, ep);
}

struct Var { const char* name; Launch f[3]; };  // waves 4/8/16
void rows_ln(const bf16* W, const bf16* X, const LnArgs& ln, int M, int N, int K, const Epi& ep, hipStream_t s) {
  gemv_rows_dispatch<X_LN>(X, ln, AttnParts{}, W, M, N, K, ep, s);
}
void rows_pl(const bf16* W, const bf16* X, const LnArgs& ln, int M, int N, int K, const Epi& ep, hipStream_t s) {
  gemv_rows_dispatch<X_PLAIN>(X, ln, AttnParts{}, W, M, N, K, ep, s);
}
template <int R, bool LN, int U>
void rl(const bf16* W, const bf16* X, const LnArgs& ln, int M, int N, int K, const Epi& ep, hipStream_t s) {
  constexpr int XM = LN ? X_LN : X_PLAIN;
  if (ep.kind == EPI_ARGMAX) { gemv_rows_launch<4, 1, XM, U>(X, ln, AttnParts{}, W, M, N, K, ep, s); return; }
  gemv_rows_launch<R, 1, XM, U>(X, ln, AttnParts{}, W, M, N, K, ep, s);
}

#define VARS(LN, NT, PF, U) {#LN "/nt" #NT "/pf" #PF "/u" #U, {lv<4, 1, LN, NT, PF, U>, lv<8, 1, LN, NT, PF, U>, lv<16, 1, LN, NT, PF, U>}}

int main(int argc, char** argv) {
  struct Shape { const char* name; int N, K; bool ln; } shapes[] = {
    {"1b1 qkv", 4608, 1536, true}, {"1b1 dense", 1536, 1536, false}, {"1b1 fc1", 6144, 1536, true},
    {"1b1 fc2", 1536, 6144, false}, {"1b1 lm_head", 250880, 1536, true},
    {"7b1 qkv", 12288, 4096, true}, {"7b1 dense", 4096, 4096, false}, {"7b1 fc1", 16384, 4096, true},
    {"7b1 fc2", 4096, 16384, false}, {"7b1 lm_head", 250880, 4096, true},
  };
  Var lnvars[] = {{"rows(LN) dispatch", {rows_ln, rows_ln, rows_ln}},
                  {"rows(LN) dispatch HOT", {rows_ln, rows_ln, rows_ln}},
                  {"rows LN R1 U2", {rl<1, true, 2>, rl<1, true, 2>, rl<1, true, 2>}},
                  {"rows LN R1 U4", {rl<1, true, 4>, rl<1, true, 4>, rl<1, true, 4>}},
                  {"rows LN R1 U8", {rl<1, true, 8>, rl<1, true, 8>, rl<1, true, 8>}},
                  {"rows LN R2 U4", {rl<2, true, 4>, rl<2, true, 4>, rl<2, true, 4>}},
                  {"rows LN R4 U4", {rl<4, true, 4>, rl<4, true, 4>, rl<4, true, 4>}}};
  Var plvars[] = {{"rows dispatch", {rows_pl, rows_pl, rows_pl}},
                  {"rows dispatch HOT", {rows_pl, rows_pl, rows_pl}},
                  {"rows R1 U2", {rl<1, false, 2>, rl<1, false, 2>, rl<1, false, 2>}},
                  {"rows R1 U4", {rl<1, false, 4>, rl<1, false, 4>, rl<1, false, 4>}},
                  {"rows R1 U8", {rl<1, false, 8>, rl<1, false, 8>, rl<1, false, 8>}},
                  {"rows R2 U4", {rl<2, false, 4>, rl<2, false, 4>, rl<2, false, 4>}},
                  {"rows R4 U4", {rl<4, false, 4>, rl<4, false, 4>, rl<4, false, 4>}}};
  const int M = argc > 1 ? atoi(argv[1]) : 1;
  size_t maxW = (size_t)250880 * 4096;
  bf16 *W, *X, *out_a; float *xf, *outf; bf16* gb; unsigned long long* keys; u32x4* sink;
  CK(hipMalloc(&W, maxW * 2)); CK(hipMalloc(&X, 32 * 16384 * 2)); CK(hipMalloc(&xf, 32 * 16384 * 4));
  CK(hipMalloc(&outf, 32 * 250880 * 4)); CK(hipMalloc(&out_a, 32 * 250880 * 2)); CK(hipMalloc(&gb, 16384 * 2 * 2));
  CK(hipMalloc(&keys, 32 * 15680 * 8)); CK(hipMalloc(&sink, 64));
  fill_rand<<<4096, 256>>>(W, maxW, 1); fill_rand<<<64, 256>>>(X, 32 * 16384, 2); fill_f<<<64, 256>>>(xf, 32 * 16384);
  fill_rand<<<64, 256>>>(gb, 2 * 16384, 3);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int REPS = 50, ROUNDS = 5;
  for (auto& sh : shapes) {
    Var* vars = sh.ln ? lnvars : plvars;
    const int nv = 2;
    const bool hot = true;
    const int ntiles = sh.N / 16, ksteps = sh.K / 32;
    int waves = 4;
    while (waves < 16 && ntiles * waves < 2048 && waves * 2 <= ksteps) waves *= 2;
    int wi = waves == 4 ? 0 : waves == 8 ? 1 : 2;
    Epi ep{}; 
    if (sh.N == 250880) { ep.kind = EPI_ARGMAX; ep.keys = keys; ep.ldo = sh.N; }
    else { ep.kind = EPI_RESID; ep.bias = gb; ep.out_f32 = outf; ep.resid = outf; ep.ldo = sh.N; }
    LnArgs ln{xf, 1, 0, gb, gb + 16384, 1e-5f};
    std::vector<std::vector<float>> t(nv + 1);
    double bytes = (double)sh.N * sh.K * 2;
    for (int r = 0; r < ROUNDS; r++) {
      for (int v = 0; v <= nv; v++) {
        for (int i = 0; i < 3; i++) {
          if (v < nv) vars[v].f[wi](W, X, ln, M, sh.N, sh.K, ep, 0);
          else stream_read<<<2048, 256>>>((const u32x4*)W, (size_t)sh.N * sh.K * 2 / 16, sink);
        }
        CK(hipEventRecord(e0));
        for (int i = 0; i < REPS; i++) {
          // rotate through 8 weight copies' worth of address space so the MALL does not serve re-reads
          const size_t nk = (size_t)sh.N * sh.K, units = (maxW - nk) / 256 + 1;
          // cycle 2 GB (no MALL reuse); the "hot" variant re-reads one copy (MALL-resident if it fits)
          const bf16* Wi = (v == nv - 1 && hot) ? W : W + (((size_t)i * (nk / 256)) % units) * 256;
          if (v < nv) vars[v].f[wi](Wi, X, ln, M, sh.N, sh.K, ep, 0);
          else stream_read<<<2048, 256>>>((const u32x4*)Wi, (size_t)sh.N * sh.K * 2 / 16, sink);
        }
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3f / REPS);
      }
    }
    printf("%-12s M=%d N=%6d K=%5d waves=%d  %.1f MB\n", sh.name, M, sh.N, sh.K, waves, bytes / 1e6);
    for (int v = 0; v <= nv; v++) {
      std::sort(t[v].begin(), t[v].end());
      const float med = t[v][ROUNDS / 2];
      printf("   %-22s median %8.2f us  min %8.2f us  %6.0f GB/s\n", v < nv ? vars[v].name : "stream_read(ref)", med,
             t[v][0], bytes / (med * 1e-6) / 1e9);
    }
  }
  CK(hipGetLastError());
  return 0;
}
