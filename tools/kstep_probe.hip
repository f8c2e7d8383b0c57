// tools/kstep_probe.hip — where a prefill GEMM K-step goes (gemm_mfma3's 128 x 128 x 64 step, 8 waves of 64 x 32
// on v_mfma_f32_32x32x16_bf16): 256 workgroups x 512 threads (one per CU) run NSTEP K-steps over a bloom-1b1 QKV
// shaped operand pair (X 512 x 1536, W 4608 x 1536: the tiles a 144-tile grid reads), with parts of the step
// switched off by template flags:
//   DMA  LDS-DMA of the step's A and B tiles (32 KB) into a 3-stage ring, counted vmcnt
//   BAR  one s_barrier per step
//   LDS  the waves' fragment reads (12 ds_read_b128 per wave per step)
//   MF   the MFMAs (8 per wave per step)
//   XCD  tile -> block mapping: blocks of one XCD (b % 8) share W column tiles (else b -> tile b % 144)
// Prints the median per-step time over blocks (s_memrealtime, 100 MHz) and the event time of the launch.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/kstep_probe.hip -o tools/kstep_probe
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int NSTEP = 48;
__device__ unsigned long long g_ks[256 * 2];
__device__ float g_sink[256 * 512];

__global__ void fill_bf(bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = d_lb32((uint32_t)i ^ seed);
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * 0.5f);
  }
}

template <bool DMA, bool BAR, bool LDS, bool MF, bool XCD>
__global__ __launch_bounds__(512) void kstep_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W, int M, int N, int K) {
  constexpr int BM = 128, BN = 128, BK = 64, NTH = 512, NSTG = 3, CA = 2, CB = 2;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTG * (BM + BN) * BK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3, r = lane & 31, h = lane >> 5;
  const int b = blockIdx.x, tiles_n = N / BN, tiles_m = M / BM;
  int t;
  if (XCD) {
    // XCD x = b % 8 owns column tiles [x * tiles_n / 8, (x + 1) * tiles_n / 8); its 32 blocks walk them x all rows
    const int x = b % 8, i = b / 8, per = tiles_n / 8;
    const int tn = x * per + (i % (per * tiles_m)) / tiles_m, tm = i % tiles_m;
    t = tm * tiles_n + tn;
  } else {
    t = b % (tiles_n * tiles_m);
  }
  const int tm = t / tiles_n, m0 = tm * BM, n0 = (t - tm * tiles_n) * BN;
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); };
  auto As = [&](int buf) { return smem + buf * (BM + BN) * BK; };
  auto Bs = [&](int buf) { return smem + buf * (BM + BN) * BK + BM * BK; };
  const __amdgpu_buffer_rsrc_t rx = attn_rsrc(X), rw = attn_rsrc(W);
  const int nk = K / BK;
  uint32_t oa[CA], ob[CB];
#pragma unroll
  for (int i = 0; i < CA; i++) {
    const int c = i * NTH + w * 64 + lane, row = c >> 3, ch = (c & 7) ^ ((row >> 1) & 7);
    oa[i] = (uint32_t)(((size_t)(m0 + row) * K + ch * 8) * 2);
    ob[i] = (uint32_t)(((size_t)(n0 + row) * K + ch * 8) * 2);
  }
  typedef __attribute__((address_space(3))) void lds_void;
  auto gload = [&](int buf, int kt) {
    const int off = (kt % nk) * BK * 2;
#pragma unroll
    for (int i = 0; i < CA; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)(As(buf) + (i * NTH + w * 64) * 8), 16, oa[i], off, 0, 0);
#pragma unroll
    for (int i = 0; i < CB; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(Bs(buf) + (i * NTH + w * 64) * 8), 16, ob[i], off, 0, 0);
  };
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int e = 0; e < 16; e++) acc[i][e] = 0.f;
  bf16x8 af[2], bfr;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int e = 0; e < 8; e++) af[i][e] = (bf16)(float)(lane + i);
#pragma unroll
  for (int e = 0; e < 8; e++) bfr[e] = (bf16)(float)(lane * 3);
  auto ktile = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < BK / 16; ks++) {
      if (LDS) {
#pragma unroll
        for (int i = 0; i < 2; i++) af[i] = *reinterpret_cast<const bf16x8*>(As(buf) + sw(wm * 64 + i * 32 + r, ks * 2 + h));
        bfr = *reinterpret_cast<const bf16x8*>(Bs(buf) + sw(wn * 32 + r, ks * 2 + h));
      }
      if (MF) {
#pragma unroll
        for (int i = 0; i < 2; i++) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr, acc[i], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; i++) acc[i][0] += (float)af[i][0] + (float)bfr[1];
      }
    }
  };
  __syncthreads();
  if (DMA) { gload(0, 0); gload(1, 1); }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int buf = 0, nbuf = NSTG - 1;
  for (int kt = 0; kt < NSTEP; kt++) {
    if (DMA) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + CB)) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (BAR) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (DMA) gload(nbuf, kt + NSTG - 1);
    ktile(buf);
    buf = buf == NSTG - 1 ? 0 : buf + 1;
    nbuf = nbuf == NSTG - 1 ? 0 : nbuf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int e = 0; e < 16; e++) s += acc[i][e];
  g_sink[b * 512 + tid] = s;
  if (tid == 0) { g_ks[b * 2] = t0; g_ks[b * 2 + 1] = t1; }
}

template <bool DMA, bool BAR, bool LDS, bool MF, bool XCD>
static void run(const char* name, const bf16* X, const bf16* W) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<double> per, ev;
  std::vector<unsigned long long> st(512);
  for (int it = 0; it < 12; it++) {
    CK(hipEventRecord(e0));
    kstep_kernel<DMA, BAR, LDS, MF, XCD><<<256, 512>>>(X, W, 512, 4608, 1536);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_ks), st.size() * 8));
    if (it < 2) continue;
    ev.push_back(ms * 1e3);
    for (int b = 0; b < 256; b++) per.push_back((st[b * 2 + 1] - st[b * 2]) * 0.01 / NSTEP);
  }
  std::sort(per.begin(), per.end()); std::sort(ev.begin(), ev.end());
  printf("%-34s per K-step p50 %.3f us  p90 %.3f us  (event %.1f us for %d steps)\n", name, per[per.size() / 2],
         per[per.size() * 9 / 10], ev[ev.size() / 2], NSTEP);
}

int main() {
  bf16 *X, *W;
  CK(hipMalloc(&X, (size_t)512 * 1536 * 2)); CK(hipMalloc(&W, (size_t)4608 * 1536 * 2));
  fill_bf<<<1024, 256>>>(X, (size_t)512 * 1536, 1); fill_bf<<<1024, 256>>>(W, (size_t)4608 * 1536, 2);
  CK(hipDeviceSynchronize());
  run<true, true, true, true, false>("full (DMA+BAR+LDS+MF)", X, W);
  run<true, true, true, true, true>("full, XCD-grouped tiles", X, W);
  run<false, true, true, true, false>("no DMA", X, W);
  run<true, false, true, true, false>("no barrier", X, W);
  run<true, true, false, true, false>("no LDS reads", X, W);
  run<true, true, true, false, false>("no MFMA", X, W);
  run<false, false, false, true, false>("MFMA only", X, W);
  run<false, false, true, false, false>("LDS reads only", X, W);
  run<true, false, false, false, false>("DMA only", X, W);
  run<true, true, false, false, false>("DMA + barrier", X, W);
  run<false, true, true, false, false>("LDS + barrier", X, W);
  run<false, true, false, true, false>("MFMA + barrier", X, W);
  return 0;
}
