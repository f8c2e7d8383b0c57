// tools/attn_stamps.hip — phase timeline of attn_prefill_tr_kernel (s_memtime stamps, ATTN_STAMPS build): per key tile
// the wait for the tile's DMA, the barrier, the next tile's DMA issue, S = K.Q^T, softmax + rescale, P packing and
// P.V issue; averaged over the blocks with the most key tiles.  Cycles of the shader clock.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -DATTN_STAMPS -I include tools/attn_stamps.hip -o tools/attn_stamps
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include "../distributed_inference_demo_amd/csrc/attn_prefill.hip"
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
int main(int argc, char** argv) {
  const int nh = 32, hd = 128, S = 512, B = 1, max_ctx = 2048;
  const int nstg = argc > 1 ? atoi(argv[1]) : 2, kgr = argc > 2 ? atoi(argv[2]) : 1;
  bf16 *q, *kc, *vc, *ctx; float *slopes, *ws; unsigned* tick; int* pastd;
  CK(hipMalloc(&q, (size_t)S * nh * hd * 2)); CK(hipMalloc(&ctx, (size_t)S * nh * hd * 2));
  CK(hipMalloc(&kc, (size_t)nh * max_ctx * hd * 2)); CK(hipMalloc(&vc, (size_t)nh * max_ctx * hd * 2));
  CK(hipMalloc(&slopes, 64 * 4)); CK(hipMalloc(&pastd, 64 * 4)); CK(hipMemset(pastd, 0, 256));
  CK(hipMalloc(&ws, 1 << 24)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  fill_rand<<<1024, 256>>>(q, (size_t)S * nh * hd, 1, 2.f); fill_rand<<<1024, 256>>>(kc, (size_t)nh * max_ctx * hd, 2, 2.f);
  fill_rand<<<1024, 256>>>(vc, (size_t)nh * max_ctx * hd, 3, 2.f);
  std::vector<float> hs(64, 0.5f);
  CK(hipMemcpy(slopes, hs.data(), 256, hipMemcpyHostToDevice));
  AttnArgs a{};
  a.q = q; a.k_cache = kc; a.v_cache = vc; a.ctx_out = ctx; a.slopes = slopes;
  a.B = B; a.S = S; a.past_dev = pastd; a.n_head = nh; a.head_dim = hd; a.max_ctx = max_ctx; a.hidden = nh * hd;
  a.inv_norm = 1.f / sqrtf((float)hd); a.pf_ws = ws; a.pf_cap = 1 << 22; a.pf_tickets = tick; a.pf_ntickets = 4096;
  a.pf_tiles = 4;
  for (int i = 0; i < 30; i++) attn_prefill_tr_launch(a, 0, nstg, 4, 256, kgr);
  CK(hipDeviceSynchronize());
  const int nb = B * nh * (S / 64);
  std::vector<unsigned long long> st((size_t)4096 * 17 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_attn_stamps), st.size() * 8));
  double ph[8] = {0}, pro = 0, epi = 0, tot = 0;
  int n = 0, ntl = 0;
  for (int b = 0; b < nb; b++) {
    const unsigned long long* s = &st[(size_t)b * 17 * 8];
    const int nt = (int)s[16 * 8 + 2];
    if (nt != 8) continue;  // (key groups: every group runs ceil(8 / KG) trips; stamps are wave 0's, group 0)
    n++;
    pro += (double)(s[0] - s[16 * 8]);
    const int trips = (nt + kgr - 1) / kgr;
    for (int it = 0; it < trips; it++) {
      const unsigned long long* t = s + it * 8;
      const unsigned long long next = it + 1 < trips ? s[(it + 1) * 8] : s[16 * 8 + 1];
      ph[0] += t[1] - t[0]; ph[1] += t[2] - t[1]; ph[2] += t[3] - t[2]; ph[3] += t[4] - t[3];
      ph[4] += t[5] - t[4]; ph[5] += t[6] - t[5]; ph[6] += next - t[6];
      ntl++;
    }
    tot += (double)(s[16 * 8 + 1] - s[16 * 8]);
  }
  const char* nm[7] = {"wait DMA", "barrier", "issue next DMA", "K.Q^T (reads+MFMA issue)", "softmax+rescale",
                       "P pack", "P.V (tr reads + MFMA) to next top"};
  printf("7b1 S512 B1, NSTG %d, key groups %d: %d blocks with 8 key tiles; cycles per loop trip (shader clock)\n", nstg, kgr, n);
  for (int i = 0; i < 7; i++) printf("  %-36s %8.0f\n", nm[i], ph[i] / ntl);
  printf("  prologue (entry -> first tile) %8.0f, whole block %8.0f cycles\n", pro / n, tot / n);
  return 0;
}
