// tools/engine_timeline.hip — in-kernel timeline of the decode engine (diagnostic build, BS_ENGINE_STAMPS):
// a bloom-1b1-shaped middle stage (24 layers, h 1536, 16 heads, B = 1, `past` cached positions, random
// weights) launched back to back like graph replays; lane 0 of each role wave stamps s_memrealtime at the
// points listed in engine.hip (ESTAMP).  Prints the launch time, per-phase segment medians over blocks and
// layers, and per hand-off the latency from the LAST producer's publish to the median / last consumer's
// "seen" stamp.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DBS_ENGINE_STAMPS tools/engine_timeline.hip -o tools/engine_timeline
#define BS_ENGINE_STAMPS 1
#include "engine/engine.hip"
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
  if (!engine_supported(0, 1, H, NH, MAXCTX)) { printf("engine not supported on this device\n"); return 1; }
  EngineArgs a{};
  a.wl = w; a.layer_stride = lb; a.kv = kv; a.kv_layer_stride = kvhalf * 2; a.kv_half = kvhalf;
  a.L = L; a.M = 1; a.h = H; a.n_head = NH; a.hd = HD; a.max_ctx = MAXCTX; a.slot = 0;
  a.eps = 1e-5f; a.inv_norm = 1.f / sqrtf((float)HD); a.slopes = slopes; a.past_dev = pastd;
  a.x_in = xin; a.x_out = xout; a.ws = ws; a.sticky_host = nullptr;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = 0; it < 5; it++) launch_decode_engine(a, 0);
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; it++) launch_decode_engine(a, 0);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned sticky = 0;
  CK(hipMemcpy(&sticky, ws + engine_status_offset(), 4, hipMemcpyDeviceToHost));
  printf("engine: %d back-to-back launches, %.1f us per launch (%.2f us per layer), past %d, sticky %u\n", iters,
         ms * 1e3 / iters, ms * 1e3 / iters / L, past, sticky);
  std::vector<unsigned long long> st((size_t)256 * 24 * 16);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_eng_stamps), st.size() * 8));
  auto S = [&](int b, int l, int k) { return (double)st[((size_t)b * 24 + l) * 16 + k]; };
  // segments inside a block (median over blocks and layers 1 .. L-2)
  struct Seg { const char* n; int k0, k1; bool s0; } segs[] = {
      {"A  LN_in (x seen -> staged)", 0, 1, false},   {"A  QKV dots (staged -> dots done)", 1, 8, false},
      {"A  QKV publish (dots -> published)", 8, 9, false}, {"B  attention (qkv seen -> record)", 5, 6, false},
      {"B  record publish (ready -> published)", 6, 10, false}, {"B  merge publish (merged -> ctx)", 7, 11, true},
      {"C  dense (ctx seen -> x1 published)", 2, 12, false}, {"D  LN+fc1 (x1 seen -> g published)", 3, 13, false},
      {"E  fc2 (g seen -> x published)", 4, 14, false}};
  for (auto& sg : segs) {
    std::vector<double> v;
    for (int l = 1; l < L - 1; l++)
      for (int b = 0; b < 256; b++) {
        if (sg.s0 && b % 16) continue;
        const double x0 = S(b, l, sg.k0), x1 = S(b, l, sg.k1);
        if (x0 > 0 && x1 >= x0) v.push_back((x1 - x0) * 0.01);
      }
    printf("%-42s p50 %6.2f p90 %6.2f us\n", sg.n, pct(v, .5), pct(v, .9));
  }
  // hand-offs: last producer publish -> consumers' seen stamps (median over layers of per-layer median / max)
  struct Edge { const char* n; int kp, kc, dl; int grp; } edges[] = {
      {"x      (fc2 -> next LN_in)", 14, 0, 1, 0}, {"q/k/v  (QKV -> attention, head)", 9, 5, 0, 1},
      {"record (attention -> merge, head)", 10, 7, 0, 2}, {"ctx    (merge -> dense)", 11, 2, 0, 0},
      {"x1     (dense -> LN_post)", 12, 3, 0, 0}, {"g      (fc1 -> fc2)", 13, 4, 0, 0}};
  for (auto& e : edges) {
    std::vector<double> med, mx;
    for (int l = 1; l < L - 2; l++) {
      for (int hg = 0; hg < (e.grp ? 16 : 1); hg++) {
        double lastp = 0;
        for (int b = 0; b < 256; b++) {
          if (e.grp && b / 16 != hg) continue;
          if (e.kp == 11 && b % 16) continue;
          lastp = std::max(lastp, S(b, l, e.kp));
        }
        std::vector<double> c;
        for (int b = 0; b < 256; b++) {
          if (e.grp && b / 16 != hg) continue;
          if (e.grp == 2 && b % 16) continue;
          const double x = S(b, l + e.dl, e.kc);
          if (x > 0) c.push_back((x - lastp) * 0.01);
        }
        if (c.empty()) continue;
        med.push_back(pct(c, .5));
        mx.push_back(pct(c, 1));
      }
    }
    printf("edge %-36s last publish -> seen: median %6.2f  last %6.2f us\n", e.n, pct(med, .5), pct(mx, .5));
  }
  // per layer: first block's x seen -> next layer's last block x seen
  std::vector<double> lay;
  for (int l = 1; l < L - 2; l++) {
    double a0 = 1e30, a1 = 0;
    for (int b = 0; b < 256; b++) { a0 = std::min(a0, S(b, l, 0)); a1 = std::max(a1, S(b, l + 1, 0)); }
    lay.push_back((a1 - a0) * 0.01);
  }
  std::vector<double> ld;
  for (int l = 1; l < L - 1; l++)
    for (int b = 0; b < 256; b++) ld.push_back((S(b, l, 15) - S(b, l - 1, 15)) * 0.01);
  printf("layer span p50 %.2f us; loader: layer issue interval p50 %.2f p90 %.2f us\n", pct(lay, .5), pct(ld, .5),
         pct(ld, .9));
  return 0;
}
