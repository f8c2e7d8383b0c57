// tools/kstep_probe2.hip — K-step structures for the prefill GEMM's 128 x 128 x 64 step (bloom-1b1 QKV operands,
// 256 workgroups, one per CU, NSTEP steps each, s_memrealtime per block):
//   NW = 8: 2 x 4 waves of 64 x 32 (gemm_mfma3's layout), NW = 4: 2 x 2 waves of 64 x 64 (a third less LDS reading:
//   A fragments shared by 2 waves instead of 4);  NSTG LDS stages;  AHEAD: the step's barrier moves to its end,
//   after the last MFMAs are issued, and guards the NEXT tile (landed for every wave), so the next step's first
//   fragments are read before the barrier's wait is over (else: barrier at the step's start, gemm_mfma3's order).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/kstep_probe2.hip -o tools/kstep_probe2
#include "../distributed_inference_demo_amd/csrc/common.h"
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int NSTEP = 48;
__device__ unsigned long long g_ks[256 * 2];
__device__ float g_sink[256 * 512];

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
}

__global__ void fill_bf(bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12;
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * 0.5f);
  }
}

template <int NW, int NSTG, bool AHEAD, bool MFONLY>
__global__ __launch_bounds__(NW * 64) void kstep2(const bf16* __restrict__ X, const bf16* __restrict__ W, int M, int N, int K) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass dropped these instantiations' stubs without a diagnostic)
  constexpr int BM = 128, BN = 128, BK = 64, NTH = NW * 64;
  constexpr int WN = NW == 8 ? 4 : 2, FI = 2, FJ = NW == 8 ? 1 : 2;  // wave grid 2 x WN; fragments per wave
  constexpr int CA = BM * BK / 8 / NTH, CB = BN * BK / 8 / NTH;       // 16-B chunks per thread per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTG * (BM + BN) * BK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN, r = lane & 31, h = lane >> 5;
  const int b = blockIdx.x, tiles_n = N / BN, tiles_m = M / BM;
  const int t = b % (tiles_n * tiles_m);
  const int tm = t / tiles_n, m0 = tm * BM, n0 = (t - tm * tiles_n) * BN;
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); };
  auto As = [&](int buf) { return smem + buf * (BM + BN) * BK; };
  auto Bs = [&](int buf) { return smem + buf * (BM + BN) * BK + BM * BK; };
  const __amdgpu_buffer_rsrc_t rx = rsrc(X), rw = rsrc(W);
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
  f32x16 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; i++)
#pragma unroll
    for (int j = 0; j < FJ; j++)
#pragma unroll
      for (int e = 0; e < 16; e++) acc[i][j][e] = 0.f;
  bf16x8 fa[2][FI], fb[2][FJ];  // fragments of ks (double-buffered by ks parity)
  auto frag = [&](int buf, int ks, int p) {
#pragma unroll
    for (int i = 0; i < FI; i++) fa[p][i] = *reinterpret_cast<const bf16x8*>(As(buf) + sw(wm * 64 + i * 32 + r, ks * 2 + h));
#pragma unroll
    for (int j = 0; j < FJ; j++) fb[p][j] = *reinterpret_cast<const bf16x8*>(Bs(buf) + sw(wn * (BN / WN) + j * 32 + r, ks * 2 + h));
  };
  auto mfma = [&](int p) {
#pragma unroll
    for (int i = 0; i < FI; i++)
#pragma unroll
      for (int j = 0; j < FJ; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][i], fb[p][j], acc[i][j], 0, 0, 0);
  };
#pragma unroll
  for (int p = 0; p < 2; p++) {
#pragma unroll
    for (int i = 0; i < FI; i++)
#pragma unroll
      for (int e = 0; e < 8; e++) fa[p][i][e] = (bf16)(float)(lane + i);
#pragma unroll
    for (int j = 0; j < FJ; j++)
#pragma unroll
      for (int e = 0; e < 8; e++) fb[p][j][e] = (bf16)(float)(lane * 3 + j);
  }
  __syncthreads();
  unsigned long long t0;
  if constexpr (MFONLY) {
    t0 = __builtin_amdgcn_s_memrealtime();
    for (int kt = 0; kt < NSTEP; kt++) {
#pragma unroll
      for (int ks = 0; ks < 4; ks++) mfma(ks & 1);
    }
  } else if constexpr (!AHEAD) {
#pragma unroll
    for (int s = 0; s < NSTG - 1; s++) gload(s, s);
    t0 = __builtin_amdgcn_s_memrealtime();
    int buf = 0, nbuf = NSTG - 1;
    for (int kt = 0; kt < NSTEP; kt++) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + CB)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      gload(nbuf, kt + NSTG - 1);
#pragma unroll
      for (int ks = 0; ks < 4; ks++) {
        frag(buf, ks, ks & 1);
        mfma(ks & 1);
      }
      buf = buf == NSTG - 1 ? 0 : buf + 1;
      nbuf = nbuf == NSTG - 1 ? 0 : nbuf + 1;
    }
  } else {
    // NSTG - 1 tiles in flight; tile 0 visible to every wave; its first fragments read
#pragma unroll
    for (int s = 0; s < NSTG - 1; s++) gload(s, s);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + CB)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    t0 = __builtin_amdgcn_s_memrealtime();
    frag(0, 0, 0);
    int buf = 0, nbuf = NSTG - 1;
    for (int kt = 0; kt < NSTEP; kt++) {
      // the stage of tile kt - 1 is free (every wave passed the last barrier after its reads of it)
      gload(nbuf, kt + NSTG - 1);
#pragma unroll
      for (int ks = 0; ks < 3; ks++) {
        frag(buf, ks + 1, (ks + 1) & 1);
        mfma(ks & 1);
      }
      mfma(1);
      // tile kt + 1 landed for this wave (NSTG - 2 younger tiles may be in flight), then for every wave
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + CB)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      buf = buf == NSTG - 1 ? 0 : buf + 1;
      nbuf = nbuf == NSTG - 1 ? 0 : nbuf + 1;
      frag(buf, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FI; i++)
#pragma unroll
    for (int j = 0; j < FJ; j++)
#pragma unroll
      for (int e = 0; e < 16; e++) s += acc[i][j][e];
  g_sink[b * 512 + tid] = s;
  if (tid == 0) { g_ks[b * 2] = t0; g_ks[b * 2 + 1] = t1; }
#endif
}

// BD: A staged by LDS-DMA as above, B (the weights) loaded by each wave straight into its MFMA fragments from
// global (16 B per lane per ks: row n0 + 32 wn + r, k 16 ks + 8 h), a register ring DB steps deep: the LDS holds A
// only (half the DMA writes, two thirds of the fragment reads); the two waves of a column pair read B twice (L2).
template <int DB>
__global__ __launch_bounds__(512) void kstep_bd(const bf16* __restrict__ X, const bf16* __restrict__ W, int M, int N, int K) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = 128, BN = 128, BK = 64, NTH = 512, NSTG = 3, CA = BM * BK / 8 / NTH;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTG * BM * BK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3, r = lane & 31, h = lane >> 5;
  const int b = blockIdx.x, tiles_n = N / BN, tiles_m = M / BM;
  const int t = b % (tiles_n * tiles_m);
  const int tm = t / tiles_n, m0 = tm * BM, n0 = (t - tm * tiles_n) * BN;
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); };
  auto As = [&](int buf) { return smem + buf * BM * BK; };
  const __amdgpu_buffer_rsrc_t rx = rsrc(X), rw = rsrc(W);
  const int nk = K / BK;
  uint32_t oa[CA];
#pragma unroll
  for (int i = 0; i < CA; i++) {
    const int c = i * NTH + w * 64 + lane, row = c >> 3, ch = (c & 7) ^ ((row >> 1) & 7);
    oa[i] = (uint32_t)(((size_t)(m0 + row) * K + ch * 8) * 2);
  }
  const uint32_t obw = (uint32_t)(((size_t)(n0 + wn * 32 + r) * K + 8 * h) * 2);
  typedef __attribute__((address_space(3))) void lds_void;
  u32x4v bq[DB][4];
  auto gload = [&](int buf, int kt) {
    const int off = (kt % nk) * BK * 2;
#pragma unroll
    for (int i = 0; i < CA; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)(As(buf) + (i * NTH + w * 64) * 8), 16, oa[i], off, 0, 0);
  };
  auto bload = [&](int slot, int kt) {
    const int off = (kt % nk) * BK * 2;
#pragma unroll
    for (int ks = 0; ks < 4; ks++) bq[slot][ks] = __builtin_amdgcn_raw_buffer_load_b128(rw, obw + ks * 32, off, 0);
  };
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int e = 0; e < 16; e++) acc[i][e] = 0.f;
  __syncthreads();
  // steps 0 .. NSTG - 2 in flight (A by DMA, B into the ring; DB == NSTG keeps the two in step)
#pragma unroll
  for (int s = 0; s < NSTG - 1; s++) { gload(s, s); bload(s, s); }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int buf = 0, nbuf = NSTG - 1;
  for (int kt = 0; kt < NSTEP; kt += DB) {
#pragma unroll
    for (int u = 0; u < DB; u++) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTG - 2) * (CA + 4)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      gload(nbuf, kt + u + NSTG - 1);
      bload((u + NSTG - 1) % DB, kt + u + NSTG - 1);
#pragma unroll
      for (int ks = 0; ks < 4; ks++) {
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; i++) af[i] = *reinterpret_cast<const bf16x8*>(As(buf) + sw(wm * 64 + i * 32 + r, ks * 2 + h));
        const bf16x8 bf = __builtin_bit_cast(bf16x8, bq[u][ks]);
#pragma unroll
        for (int i = 0; i < 2; i++) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf, acc[i], 0, 0, 0);
      }
      buf = buf == NSTG - 1 ? 0 : buf + 1;
      nbuf = nbuf == NSTG - 1 ? 0 : nbuf + 1;
    }
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
#endif
}

static void run_bd(const char* name, const bf16* X, const bf16* W) {
  std::vector<double> per;
  std::vector<unsigned long long> st(512);
  for (int it = 0; it < 12; it++) {
    kstep_bd<3><<<256, 512>>>(X, W, 512, 4608, 1536);
    CK(hipDeviceSynchronize());
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_ks), st.size() * 8));
    if (it < 2) continue;
    for (int b = 0; b < 256; b++) per.push_back((st[b * 2 + 1] - st[b * 2]) * 0.01 / NSTEP);
  }
  std::sort(per.begin(), per.end());
  printf("%-44s per K-step p50 %.3f us  p90 %.3f us\n", name, per[per.size() / 2], per[per.size() * 9 / 10]);
}

template <int NW, int NSTG, bool AHEAD, bool MFONLY>
static void run(const char* name, const bf16* X, const bf16* W) {
  std::vector<double> per;
  std::vector<unsigned long long> st(512);
  for (int it = 0; it < 12; it++) {
    kstep2<NW, NSTG, AHEAD, MFONLY><<<256, NW * 64>>>(X, W, 512, 4608, 1536);
    CK(hipDeviceSynchronize());
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_ks), st.size() * 8));
    if (it < 2) continue;
    for (int b = 0; b < 256; b++) per.push_back((st[b * 2 + 1] - st[b * 2]) * 0.01 / NSTEP);
  }
  std::sort(per.begin(), per.end());
  printf("%-44s per K-step p50 %.3f us  p90 %.3f us\n", name, per[per.size() / 2], per[per.size() * 9 / 10]);
}

int main() {
  bf16 *X, *W;
  CK(hipMalloc(&X, (size_t)512 * 1536 * 2)); CK(hipMalloc(&W, (size_t)4608 * 1536 * 2));
  fill_bf<<<1024, 256>>>(X, (size_t)512 * 1536, 1); fill_bf<<<1024, 256>>>(W, (size_t)4608 * 1536, 2);
  CK(hipDeviceSynchronize());
  run<8, 3, false, false>("8 waves 64x32, 3 stages (gemm_mfma3)", X, W);
  run_bd("8 waves 64x32, A by DMA, B direct to registers", X, W);
  run<8, 3, true, false>("8 waves 64x32, 3 stages, ahead", X, W);
  run<8, 4, true, false>("8 waves 64x32, 4 stages, ahead", X, W);
  run<4, 3, false, false>("4 waves 64x64, 3 stages", X, W);
  run<4, 3, true, false>("4 waves 64x64, 3 stages, ahead", X, W);
  run<4, 4, true, false>("4 waves 64x64, 4 stages, ahead", X, W);
  run<8, 3, false, true>("8 waves MFMA only", X, W);
  run<4, 3, false, true>("4 waves MFMA only", X, W);
  return 0;
}
