// tools/engine_timeline.hip — in-kernel timeline of the decode engine (diagnostic build, BS_ENGINE_STAMPS):
// a bloom-1b1-shaped middle stage (24 layers, h 1536, 16 heads, B = 1, 580 cached positions, random
// weights) launched back to back like graph replays; wave 0 of every block stamps s_memrealtime at five
// points of each phase (start, input seen, S2 = activations staged, S3 = dots done, published; phase B:
// start, q/k/v seen, attention done, split record published, head merged).
// Prints per phase the median/p90 over blocks and layers of each segment, and per edge the latency from
// the LAST producer's publish to the FIRST / median consumer's edge-seen stamp.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DBS_ENGINE_STAMPS tools/engine_timeline.hip -o tools/engine_timeline
#define BS_ENGINE_STAMPS 1
#include "../distributed_inference_demo_amd/csrc/engine.hip"
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

static double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[(size_t)std::min<double>(v.size() - 1, q * (v.size() - 1) + 0.5)];
}

int main(int argc, char** argv) {
  const int L = 24, H = 1536, NH = 16, HD = 96, MAXCTX = 1024;
  const int past = argc > 1 ? atoi(argv[1]) : 580;
  const size_t lb = engine_layer_bytes(H);
  char* w; CK(hipMalloc(&w, lb * L));
  fill_rand<<<4096, 256>>>((bf16*)w, lb * L / 2, 7, 0.04f);
  // LayerNorm gammas near 1 (beta ~0): overwrite with 1.0 so the rows stay well scaled
  std::vector<bf16> ones(H, (bf16)1.0f);
  for (int l = 0; l < L; l++) {
    CK(hipMemcpy(w + l * lb + LayerOff<1536>::LN1_G, ones.data(), H * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(w + l * lb + LayerOff<1536>::LN2_G, ones.data(), H * 2, hipMemcpyHostToDevice));
  }
  const size_t kvhalf = (size_t)NH * MAXCTX * HD * 2;
  char* kv; CK(hipMalloc(&kv, kvhalf * 2 * L)); CK(hipMemset(kv, 0, kvhalf * 2 * L));
  char* ws; const size_t wsb = engine_ws_bytes(H, NH); CK(hipMalloc(&ws, wsb)); CK(hipMemset(ws, 0, wsb));
  float *xin, *xout, *slopes; int* pastd;
  CK(hipMalloc(&xin, H * 4)); CK(hipMalloc(&xout, H * 4)); CK(hipMalloc(&slopes, NH * 4)); CK(hipMalloc(&pastd, 64));
  std::vector<float> hx(H), hs(NH);
  for (int i = 0; i < H; i++) hx[i] = (float)((i * 37) % 101) / 50.f - 1.f;
  for (int i = 0; i < NH; i++) hs[i] = powf(2.f, -8.f * (i + 1) / NH);
  CK(hipMemcpy(xin, hx.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(slopes, hs.data(), NH * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(pastd, &past, 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  EngineArgs a{};
  a.wl = w; a.layer_stride = lb; a.kv = kv; a.kv_layer_stride = kvhalf * 2; a.kv_half = kvhalf;
  a.L = L; a.M = 1; a.h = H; a.n_head = NH; a.hd = HD; a.max_ctx = MAXCTX; a.slot = 0;
  a.eps = 1e-5f; a.inv_norm = 1.f / sqrtf((float)HD); a.slopes = slopes; a.past_dev = pastd;
  a.x_in = xin; a.x_out = xout; a.ws = ws;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; it++) launch_decode_engine(a, 0);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("engine: %d back-to-back launches, %.1f us per launch (%.2f us per layer), past %d\n", iters, ms * 1e3 / iters,
         ms * 1e3 / iters / L, past);
  std::vector<unsigned long long> st((size_t)256 * 64 * 5 * 6);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_eng_stamps), st.size() * 8));
  auto S = [&](int b, int l, int ph, int k) { return st[(((size_t)b * 64 + l) * 5 + ph) * 6 + k]; };
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < 256; b++) { t0 = std::min(t0, S(b, 0, 0, 0)); tend = std::max(tend, S(b, L - 1, 4, 4)); }
  printf("stamped span (first A start -> last E publish): %.2f us\n", (tend - t0) * 0.01);
  const char* names[5] = {"A ln+qkv", "B attn", "C dense", "D ln+fc1", "E fc2"};
  const char* seg[4] = {"wait", "stage", "dots", "publish"};
  const char* segb[4] = {"wait", "attn", "record", "merge"};
  for (int ph = 0; ph < 5; ph++) {
    printf("%-9s", names[ph]);
    for (int k = 0; k < 4; k++) {
      std::vector<double> v;
      for (int l = 1; l < L - 1; l++)
        for (int b = 0; b < 256; b++) {
          const unsigned long long x0 = S(b, l, ph, k), x1 = S(b, l, ph, k + 1);
          if (x0 && x1 && x1 >= x0) v.push_back((x1 - x0) * 0.01);
        }
      printf(" | %-7s p50 %5.2f p90 %5.2f", ph == 1 ? segb[k] : seg[k], pct(v, .5), pct(v, .9));
    }
    printf("\n");
  }
  // per layer: span of each phase from the first block's start to the last block's publish
  std::vector<double> layer_us;
  for (int l = 1; l < L - 1; l++) {
    unsigned long long a0 = ~0ull, a1 = 0;
    for (int b = 0; b < 256; b++) { a0 = std::min(a0, S(b, l, 0, 0)); a1 = std::max(a1, S(b, l + 1, 0, 0)); }
    layer_us.push_back((a1 - a0) * 0.01);
  }
  printf("layer (A start of first block -> next layer's last A start): p50 %.2f us\n", pct(layer_us, .5));
  // edges: last publish of the producing phase -> consumers' edge-seen stamps
  struct Edge { const char* n; int pph, cph, dl; } edges[] = {{"QKV->attn", 0, 1, 0}, {"X1->LN2", 2, 3, 0}, {"G->fc2", 3, 4, 0},
                                                            {"X2->next A", 4, 0, 1}, {"CTX->dense", 1, 2, 0}};
  for (auto& e : edges) {
    std::vector<double> first, med, lastc;
    for (int l = 1; l < L - 2; l++) {
      unsigned long long lastp = 0;
      for (int b = 0; b < 256; b++) lastp = std::max(lastp, S(b, l, e.pph, 4));
      std::vector<double> c;
      for (int b = 0; b < 256; b++) {
        const unsigned long long x = S(b, l + e.dl, e.cph, 1);
        if (x) c.push_back(((double)x - (double)lastp) * 0.01);
      }
      if (c.empty()) continue;
      first.push_back(pct(c, 0)); med.push_back(pct(c, .5)); lastc.push_back(pct(c, 1));
    }
    printf("edge %-11s last publish -> seen: first %.2f  median %.2f  last %.2f us\n", e.n, pct(first, .5), pct(med, .5),
           pct(lastc, .5));
  }
  return 0;
}
