// tools/gemm_splitk_bench.hip — prefill GEMM variants on the BLOOM prefill shapes (M tokens x N x K), HIP events
// around 20 back-to-back launches (median of 7): the library's dispatch (launch_linear), the round-2 tiles (64x64 / 64x32, 4-deep
// ring) and 128x128 tiles with split-K KS = 1, 2, 3, 4, 6.  Every split-K output is checked against KS = 1 (the
// same products summed in another order: max relative difference printed); gemm_mfma3 (128x128 tiles on
// v_mfma_f32_32x32x16_bf16, stream-K) at the dispatch's grid with and without the XCD-aware placement (XM), and at
// grids of 192..512 blocks.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm_splitk_bench.hip
//        distributed_inference_demo_amd/csrc/attn_prefill.hip -o tools/gemm_splitk_bench
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = d_lb32((uint32_t)i ^ seed);
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * 0.5f);
  }
}

int main() {
  struct Sh { const char* name; int M, N, K; } shapes[] = {
      {"1b1 qkv", 512, 4608, 1536}, {"1b1 dense", 512, 1536, 1536}, {"1b1 fc1", 512, 6144, 1536},
      {"1b1 fc2", 512, 1536, 6144}, {"7b1 qkv", 512, 12288, 4096}, {"7b1 dense", 512, 4096, 4096},
      {"7b1 fc1", 512, 16384, 4096}, {"7b1 fc2", 512, 4096, 16384}, {"3b dense B2", 1024, 2560, 2560},
      // long prompts / batched prefill: >= 512 tiles (the 2-stage, two-blocks-per-CU question)
      {"7b1 qkv 2k", 2048, 12288, 4096}, {"7b1 fc1 1k", 1024, 16384, 4096}, {"7b1 dense 2k", 2048, 4096, 4096},
      {"1b1 fc1 4k", 4096, 6144, 1536}, {"1b1 qkv 4k", 4096, 4608, 1536},
      // bloom-1b1 at 1024 / 2048 tokens (288..1536 tiles: where whole-tile grids of 384 / 512 blocks might apply)
      {"1b1 qkv 1k", 1024, 4608, 1536}, {"1b1 fc1 1k", 1024, 6144, 1536}, {"1b1 fc2 1k", 1024, 1536, 6144},
      {"1b1 qkv 2k", 2048, 4608, 1536}, {"1b1 fc1 2k", 2048, 6144, 1536}, {"1b1 fc2 2k", 2048, 1536, 6144},
      // round 6: configs[4]'s prefills (16 rows x 256 .. 1024 tokens per micro-batch at N = 1), 256 x 256 tiles
      {"7b1 qkv 4k", 4096, 12288, 4096}, {"7b1 dense 4k", 4096, 4096, 4096}, {"7b1 fc1 4k", 4096, 16384, 4096},
      {"7b1 fc2 4k", 4096, 4096, 16384}, {"7b1 qkv 16k", 16384, 12288, 4096}, {"7b1 fc1 16k", 16384, 16384, 4096},
      {"7b1 fc2 16k", 16384, 4096, 16384}, {"7b1 dense 16k", 16384, 4096, 4096}, {"7b1 fc2 8k", 8192, 4096, 16384},
      {"7b1 qkv 3840", 3840, 12288, 4096}, {"7b1 dense 3840", 3840, 4096, 4096}, {"3b qkv 4k", 4096, 7680, 2560},
      {"3b fc1 4k", 4096, 10240, 2560}, {"3b fc2 4k", 4096, 2560, 10240}};
  const char* only = getenv("GSB_ONLY");  // substring filter on the shape names
  bf16 *X, *W, *bias; float *out, *ref, *resid, *ws; unsigned* tick;
  const size_t MMAX = 16384;
  CK(hipMalloc(&X, MMAX * 16384 * 2)); CK(hipMalloc(&W, (size_t)16384 * 16384 * 2));
  CK(hipMalloc(&bias, 65536 * 2)); CK(hipMalloc(&out, MMAX * 16384 * 4)); CK(hipMalloc(&ref, MMAX * 16384 * 4));
  CK(hipMalloc(&resid, MMAX * 16384 * 4)); CK(hipMemset(resid, 0, MMAX * 16384 * 4));
  const size_t cap = (size_t)1024 * 128 * 128;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  fill_rand<<<4096, 256>>>(X, MMAX * 16384, 1); fill_rand<<<4096, 256>>>(W, (size_t)16384 * 16384, 2);
  fill_rand<<<64, 256>>>(bias, 65536, 3);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    if (only && !strstr(sh.name, only)) continue;
    const int M = sh.M, N = sh.N, K = sh.K;
    Epi ep{};
    ep.kind = EPI_RESID; ep.bias = bias; ep.out_f32 = out; ep.resid = resid; ep.ldo = N;
    ep.sk_ws = ws; ep.sk_tickets = tick; ep.sk_cap = cap; ep.sk_ntickets = 4096;
    // per launch: 20 launches back to back between two events (as tools/gemm_shapes_torch.py times hipBLASLt:
    // a lone launch between events also counts the ~5 us the events add), median of 7 such runs
    auto timeit = [&](auto&& fn) {
      std::vector<float> t;
      for (int i = 0; i < 5; i++) fn();
      for (int it = 0; it < 7; it++) {
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; i++) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3f / 20);
      }
      std::sort(t.begin(), t.end());
      return t[t.size() / 2];
    };
    const double fl = 2.0 * M * N * K;
    auto line = [&](const char* v, float us) {
      printf("%-10s M=%4d N=%5d K=%5d  %-22s %8.2f us  %6.1f TFLOP/s  %.3f of 2500\n", sh.name, M, N, K, v, us,
             fl / us * 1e-6, fl / us * 1e-6 / 2500);
    };
    line("launch_linear", timeit([&] { launch_linear(1, X, W, M, N, K, ep, 0); }));
    // reference output: 64x32, KS = 1
    gemm2_launch<64, 32, 4>(X, W, M, N, K, ep, 0, 1);
    CK(hipMemcpy(ref, out, (size_t)M * N * 4, hipMemcpyDeviceToDevice));
    std::vector<float> hr((size_t)M * N), ho((size_t)M * N);
    CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
    auto variant = [&](const char* tile, int bm, int bn, int ks, auto&& fn) {
      const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
      if (K % (ks * 64) || (size_t)tiles * ks * bm * bn > cap || tiles > 4096) return;
      char nm[64];
      snprintf(nm, sizeof nm, "%s KS=%d (%ld)", tile, ks, tiles * ks);
      const float us = timeit(fn);
      CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
      line(nm, us);
      if (md > 1e-4) printf("           MISMATCH max |diff| %.3g\n", md);
    };
    // every shape with >= 256 whole 256 x 256 tiles, whether or not the library's dispatch takes them (threshold sweep)
    const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
    if (const int gb = (K % 64 == 0 && t256 >= 256) ? (int)t256 : 0) {
      char nm[64];
      snprintf(nm, sizeof nm, "m32 256x256 G=%d", gb);
      const float us = timeit([&] { gemm3_launch<2, true, 256, 256>(X, W, M, N, K, ep, 0, gb); });
      CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
      line(nm, us);
      printf("           max |diff| vs 64x32 %.3g%s\n", md, md > 1e-3 ? "  MISMATCH" : "");
    }
    if (M > 4096) continue;  // the big shapes: the library and the 256 x 256 tiles only
    for (int ks : {1, 4})
      variant("64x64 r4", 64, 64, ks, [&] { gemm2_launch<64, 64, 4>(X, W, M, N, K, ep, 0, ks); });
    if (const int G = gemm3_grid(M, N, K, ep)) {
      for (int xm = 0; xm < 2; xm++) {
        char nm[64];
        snprintf(nm, sizeof nm, "m32 dispatch G=%d XM=%d", G, xm);
        const float us = timeit([&] {
          if (xm) gemm3_launch<3, true>(X, W, M, N, K, ep, 0, G);
          else gemm3_launch<3, false>(X, W, M, N, K, ep, 0, G);
        });
        CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
        line(nm, us);
        if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
      }
    }
    if (M <= 1024 && N <= 6144) {  // 128 x 96 stream-K at fixed grids on every small shape (round 5)
      for (int g2 : {128, 192, 256}) {
        char nm[64];
        snprintf(nm, sizeof nm, "m32 128x96 SKall G=%d", g2);
        const float u2 = timeit([&] { gemm3_launch<3, true, 96>(X, W, M, N, K, ep, 0, g2); });
        CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
        line(nm, u2);
        if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
      }
    }
    if (const int gn = gemm3_n96_grid(M, N, K, ep)) {
      char nm[64];
      snprintf(nm, sizeof nm, "m32 128x96 G=%d", gn);
      const float us = timeit([&] { gemm3_launch<3, true, 96>(X, W, M, N, K, ep, 0, gn); });
      CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
      line(nm, us);
      if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
      for (int g2 : {192, 256}) {  // stream-K over 128 x 96 tiles
        snprintf(nm, sizeof nm, "m32 128x96 SK G=%d", g2);
        const float u2 = timeit([&] { gemm3_launch<3, true, 96>(X, W, M, N, K, ep, 0, g2); });
        CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
        md = 0;
        for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
        line(nm, u2);
        if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
      }
    }
    if (const int gw = gemm3_wide_grid(M, N, K, ep)) {
      char nm[64];
      snprintf(nm, sizeof nm, "m32 wide 128x256 G=%d", gw);
      const float us = timeit([&] { gemm3_launch<3, true, 256>(X, W, M, N, K, ep, 0, gw); });
      CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
      line(nm, us);
      if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
    }
    for (int v = 0; v < 6; v++) {
      const int G = v < 3 ? (int[]){192, 256, 384}[v] : (int[]){256, 384, 512}[v - 3];
      const int nst = v < 3 ? 3 : 2;
      char nm[64];
      snprintf(nm, sizeof nm, "m32 %dstg G=%d", nst, G);
      const float us = timeit([&] {
        if (nst == 3) gemm3_launch<3>(X, W, M, N, K, ep, 0, G);
        else gemm3_launch<2>(X, W, M, N, K, ep, 0, G);
      });
      CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < ho.size(); i++) md = std::max(md, (double)fabsf(ho[i] - hr[i]));
      line(nm, us);
      if (md > 1e-3) printf("           MISMATCH max |diff| %.3g\n", md);
    }
  }
  return 0;
}
