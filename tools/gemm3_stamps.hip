// tools/gemm3_stamps.hip — where a gemm_mfma3 block spends its time (diagnostic build, GEMM3_STAMPS): every block
// records s_memrealtime (100 MHz) at entry, after its first segment's first tile is staged, after that segment's K loop and at exit (its
// stores drained); printed per shape: the span from the first entry to the last exit beside the HIP-event time,
// the entry spread (dispatch ramp), and the median prologue / K loop / epilogue (split-K reduction included).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm3_stamps.hip -o tools/gemm3_stamps
#define GEMM3_STAMPS 1
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = d_lb32((uint32_t)i ^ seed);
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * 0.5f);
  }
}

static double med(std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0 : v[v.size() / 2]; }

int main() {
  struct Sh { const char* name; int M, N, K, G, kind; } shapes[] = {
      {"1b1 qkv", 512, 4608, 1536, 144, EPI_RESID}, {"1b1 fc1", 512, 6144, 1536, 192, EPI_GELU},
      {"1b1 fc2 KS=4", 512, 1536, 6144, 192, EPI_RESID}, {"7b1 qkv", 512, 12288, 4096, 384, EPI_RESID},
      {"7b1 fc2 KS=2", 512, 4096, 16384, 256, EPI_RESID}};
  bf16 *X, *W, *bias, *act; float *out, *resid, *ws; unsigned* tick;
  CK(hipMalloc(&X, (size_t)1024 * 16384 * 2)); CK(hipMalloc(&W, (size_t)16384 * 16384 * 2));
  CK(hipMalloc(&bias, 65536 * 2)); CK(hipMalloc(&out, (size_t)1024 * 16384 * 4)); CK(hipMalloc(&act, (size_t)1024 * 16384 * 2));
  CK(hipMalloc(&resid, (size_t)1024 * 16384 * 4)); CK(hipMemset(resid, 0, (size_t)1024 * 16384 * 4));
  const size_t cap = (size_t)1024 * 128 * 128;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  fill_rand<<<4096, 256>>>(X, (size_t)1024 * 16384, 1); fill_rand<<<4096, 256>>>(W, (size_t)16384 * 16384, 2);
  fill_rand<<<64, 256>>>(bias, 65536, 3);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<unsigned long long> st(4096 * 4);
  for (auto& sh : shapes) {
    Epi ep{};
    ep.kind = sh.kind; ep.bias = bias; ep.out_f32 = out; ep.out_act = act; ep.resid = resid; ep.ldo = sh.N;
    ep.sk_ws = ws; ep.sk_tickets = tick; ep.sk_cap = cap; ep.sk_ntickets = 4096;
    std::vector<double> ev, span, ramp, pro, loop, epi;
    for (int it = 0; it < 15; it++) {
      CK(hipEventRecord(e0)); gemm3_launch(X, W, sh.M, sh.N, sh.K, ep, 0, sh.G); CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_gemm3_stamps), st.size() * 8));
      if (it < 5) continue;
      const int nb = sh.G;
      unsigned long long a0 = ~0ull, a1 = 0, amax0 = 0;
      for (int b = 0; b < nb; b++) {
        const unsigned long long* s = &st[b * 4];
        a0 = std::min(a0, s[0]); amax0 = std::max(amax0, s[0]); a1 = std::max(a1, s[3]);
        pro.push_back((s[1] - s[0]) * 0.01); loop.push_back((s[2] - s[1]) * 0.01); epi.push_back((s[3] - s[2]) * 0.01);
      }
      ev.push_back(ms * 1e3); span.push_back((a1 - a0) * 0.01); ramp.push_back((amax0 - a0) * 0.01);
    }
    printf("%-18s M=%4d N=%5d K=%5d G=%d  event %6.2f us  span %6.2f  entry ramp %5.2f | prologue %5.2f  K loop %6.2f  "
           "epilogue %5.2f (block medians)\n", sh.name, sh.M, sh.N, sh.K, sh.G, med(ev), med(span), med(ramp), med(pro),
           med(loop), med(epi));
  }
  return 0;
}
