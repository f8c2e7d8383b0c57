// tools/gemv_timeline.hip — in-kernel timeline of the decode GEMVs (diagnostic build, BS_STAMPS):
// per block, s_memrealtime at entry / after the prologue (LayerNorm) / after the K loop / after the
// epilogue, for one cold launch (weights rotated through 2 GB) of each bloom-1b1 decode GEMV shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DBS_STAMPS tools/gemv_timeline.hip -o tools/gemv_timeline
#define BS_STAMPS 1
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
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

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)std::min<double>(v.size() - 1, q * (v.size() - 1) + 0.5)];
}

int main() {
  const size_t maxW = (size_t)1 << 30;
  bf16 *W, *X, *gb, *act; float *xf, *outf; int* pastd;
  CK(hipMalloc(&W, maxW * 2)); CK(hipMalloc(&X, 16384 * 2)); CK(hipMalloc(&xf, 16384 * 4));
  CK(hipMalloc(&outf, 65536 * 4)); CK(hipMalloc(&gb, 16384 * 2 * 2)); CK(hipMalloc(&act, 65536 * 2));
  bf16* kv; CK(hipMalloc(&kv, (size_t)2 * 16 * 1024 * 128 * 2)); CK(hipMalloc(&pastd, 64));
  CK(hipMemset(pastd, 0, 64));
  fill_rand<<<4096, 256>>>(W, maxW, 1); fill_rand<<<64, 256>>>(X, 16384, 2); fill_f<<<64, 256>>>(xf, 16384);
  fill_rand<<<64, 256>>>(gb, 2 * 16384, 3);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Shape { const char* name; int N, K, kind; bool ln; } shapes[] = {
    {"1b1 qkv LN", 4608, 1536, EPI_QKV, true}, {"1b1 dense", 1536, 1536, EPI_RESID, false},
    {"1b1 fc1 LN", 6144, 1536, EPI_GELU, true}, {"1b1 fc2", 1536, 6144, EPI_RESID, false},
    {"1b1 qkv plain", 4608, 1536, EPI_QKV, false}};
  for (auto& sh : shapes) {
    const int N = sh.N, K = sh.K;
    Epi ep{};
    ep.kind = sh.kind; ep.bias = gb; ep.ldo = N;
    ep.out_f32 = outf; ep.resid = outf; ep.out_act = act;
    ep.q_out = act; ep.k_cache = kv; ep.v_cache = kv + (size_t)16 * 1024 * 128;
    ep.hidden = 1536; ep.head_dim = 96; ep.max_ctx = 1024; ep.n_head = 16; ep.seq = 1; ep.slot = 0; ep.past_dev = pastd;
    LnArgs ln{xf, 1, 0, gb, gb + 16384, 1e-5f};
    const size_t nk = (size_t)N * K, rot = (maxW - nk) / 256 + 1;
    const bool fc2 = sh.name[4] == 'f' && sh.name[6] == '2';
    int R, waves;
    rows_geometry(N, K, 1, fc2 ? 1 : 2, &R, &waves);
    const int nb = (N + waves * R - 1) / (waves * R);
    for (int it = 0; it < 12; it++) {
      const bf16* w = W + (((size_t)it * (nk / 256 + 7)) % rot) * 256;
      CK(hipEventRecord(e0));
      if (sh.ln) gemv_rows_dispatch<X_LN>(nullptr, ln, AttnParts{}, w, 1, N, K, ep, 0);
      else gemv_rows_dispatch<X_PLAIN>(X, ln, AttnParts{}, w, 1, N, K, ep, 0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      if (it < 11) continue;
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> st(nb * 4);
      CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
      unsigned long long t0 = ~0ull, tend = 0;
      for (int b = 0; b < nb; b++) { t0 = std::min(t0, st[b * 4]); tend = std::max(tend, st[b * 4 + 3]); }
      std::vector<double> start, pro, loop, epi, end;
      for (int b = 0; b < nb; b++) {
        start.push_back((st[b * 4] - t0) * 0.01); pro.push_back((st[b * 4 + 1] - st[b * 4]) * 0.01);
        loop.push_back((st[b * 4 + 2] - st[b * 4 + 1]) * 0.01); epi.push_back((st[b * 4 + 3] - st[b * 4 + 2]) * 0.01);
        end.push_back((st[b * 4 + 3] - t0) * 0.01);
      }
      printf("%-14s N=%5d K=%5d R=%d waves=%2d blocks %4d  event %.2f us  span(first start -> last epilogue) %.2f us\n", sh.name, N, K, R, waves,
             nb, ms * 1e3, (tend - t0) * 0.01);
      printf("   start  p50 %.2f p90 %.2f max %.2f | prologue p50 %.2f p90 %.2f | K loop p50 %.2f p90 %.2f max %.2f | "
             "epilogue p50 %.2f | end p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
             pct(start, .5), pct(start, .9), pct(start, 1), pct(pro, .5), pct(pro, .9), pct(loop, .5), pct(loop, .9),
             pct(loop, 1), pct(epi, .5), pct(end, .1), pct(end, .5), pct(end, .9), pct(end, 1));
    }
  }
  return 0;
}
