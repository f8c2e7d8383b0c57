// tools/rows8_bench.hip — batched decode GEMVs at M = 5..8 rows: gemv_rows8_kernel (below: LayerNorm / activations
// staged by LDS-DMA in the GEMV's prologue) against the library's path (ln_rows_wave_kernel + gemv_ldsw4 / tiles) on the
// BLOOM block shapes.  Time = 20 back-to-back launches between HIP events / 20, median of 7 groups.  Outputs of the
// two paths are compared (max |diff| of the bf16 GELU epilogue outputs).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/rows8_bench.hip -o tools/rows8_bench
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <algorithm>

// The experiment (round 5, measured slower than the round-4 path on every shape: profiles/r05_rows8_ab.txt; kept
// here, out of the library):
// gemv_rows8: batched decode GEMV for 4 < M <= 8 rows (round 5), the rows kernel's streaming
// geometry (a wave owns R whole weight rows, 1-KB loads of one row per instruction, U 512-column chunks in
// flight, one block of up to 16 waves per CU, every CU the same weight bytes) with the activations staged
// once per block in LDS:
//  * LN (QKV, fc1): the fp32 rows arrive by LDS-DMA (buffer_load ... lds, wave w DMAs rows w, w + nw, ...)
//    together with gamma / beta, all issued BEFORE the weight stream, so waiting for them (a counted vmcnt)
//    leaves the weights in flight; each wave then normalises its own rows in place (shifted-sum statistics
//    with c = the row's first element, as ln_rows_finish; fp32 -> bf16 written over the row's first half,
//    in increasing chunk order so no unread value is overwritten).  No LayerNorm launch.
//  * PLAIN (dense, fc2): the bf16 rows by LDS-DMA the same way.
//  * dot products on v_dot2 (8 rows x R per 16-B X read from LDS, shared by the wave's R rows); wave
//    reductions; lane j = 8 r + m stores (row r, token m).
// X bytes per block: LN M x K x 4 + 4 K (<= 144 KB at K = 4096), PLAIN M x K x 2 (<= 128 KB).
// ------------------------------------------------------------------------------------
template <int R, int U, bool LN>
__global__ __launch_bounds__(1024) void gemv_rows8_kernel(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                                          LnArgs ln, int M, int N, int K, Epi ep) {
  constexpr int MM = 8;
  typedef __attribute__((address_space(3))) void lds_void;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n0 = (blockIdx.x * nw + w) * R;
  const int er = lane >> 3, em = lane & 7;
  const EpiPre pre = epi_prefetch<bf16>(ep, em, n0 + er, er < R && em < M && n0 + er < N);
  // activations by LDS-DMA: row m of the block's image at m * rb bytes; LN: gamma, beta after the rows
  const int rb = LN ? K * 4 : K * 2, npc = rb >> 10;  // bytes per row, 1-KB pieces per row
  {
    const __amdgpu_buffer_rsrc_t rx = LN ? __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ln.x), (short)0, 0x7FFFFFFF, 0x00020000)
                                         : __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(X), (short)0, 0x7FFFFFFF, 0x00020000);
    for (int m = w; m < M; m += nw) {
      const int src_row = LN ? m * ln.row_stride + ln.row_offset : m;
      const int so = src_row * rb;
      for (int pc = 0; pc < npc; pc++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)(smem + m * rb + pc * 1024), 16, lane * 16 + pc * 1024, so, 0, 0);
    }
    if (LN && w == nw - 1) {  // gamma, beta: K x 2 bytes each
      const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(ln.gamma), (short)0, K * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t rbb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(ln.beta), (short)0, K * 2, 0x00020000);
      for (int pc = 0; pc < (K * 2) >> 10; pc++) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (lds_void*)(smem + M * rb + pc * 1024), 16, lane * 16 + pc * 1024, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rbb, (lds_void*)(smem + M * rb + K * 2 + pc * 1024), 16, lane * 16 + pc * 1024, 0, 0, 0);
      }
    }
  }
  asm volatile("" ::: "memory");  // the weight loads stay behind the activation DMAs (the counted wait below)
  __builtin_amdgcn_sched_barrier(0);
  const bf16* wr[R];
#pragma unroll
  for (int r = 0; r < R; r++) wr[r] = W + (size_t)min(n0 + r, N - 1) * K;
  bf16x8 wv[U][R];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int k = min(u * 512 + lane * 8, K - 8);
#pragma unroll
    for (int r = 0; r < R; r++) wv[u][r] = wload<true>(wr[r] + k);
  }
  // this wave's activation DMAs (older than the weights) have landed
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * R) : "memory");
  __builtin_amdgcn_s_barrier();  // every wave's rows (and gamma / beta) are in LDS
  asm volatile("" ::: "memory");
  if constexpr (LN) {
    const float invk = 1.0f / (float)K;
    const bf16* gs = reinterpret_cast<const bf16*>(smem + M * rb);
    const bf16* bs = gs + K;
    for (int m = w; m < M; m += nw) {
      float* xr = reinterpret_cast<float*>(smem + m * rb);
      const float c = xr[0];
      float a1 = 0.f, a2 = 0.f;
      for (int k = lane * 4; k < K; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + k);
        const float d0 = v.x - c, d1 = v.y - c, d2 = v.z - c, d3 = v.w - c;
        a1 += (d0 + d1) + (d2 + d3);
        a2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
      const float t1 = wave_sum(a1) * invk, t2 = wave_sum(a2) * invk;
      const float mean = c + t1, rstd = 1.0f / sqrtf(fmaxf(t2 - t1 * t1, 0.f) + ln.eps);
      bf16* xo = reinterpret_cast<bf16*>(xr);  // in place: chunk j's bf16 lands on bytes chunk j / 2 held
      for (int k = lane * 4; k < K; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + k);
        float4 g, bb;
        bf16x4_to_f32(*reinterpret_cast<const uint2*>(gs + k), g);
        bf16x4_to_f32(*reinterpret_cast<const uint2*>(bs + k), bb);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 o;
        o[0] = (bf16)((v.x - mean) * rstd * g.x + bb.x);
        o[1] = (bf16)((v.y - mean) * rstd * g.y + bb.y);
        o[2] = (bf16)((v.z - mean) * rstd * g.z + bb.z);
        o[3] = (bf16)((v.w - mean) * rstd * g.w + bb.w);
        *reinterpret_cast<bf16x4*>(xo + k) = o;  // after this chunk's read (a wave's LDS ops run in order)
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  const bf16* xs = reinterpret_cast<const bf16*>(smem);
  const int xstride = rb / 2;  // bf16 elements between rows
  float acc[R][MM];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int m = 0; m < MM; m++) acc[r][m] = 0.f;
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  for (int kb = 0; kb < K; kb += 512 * U) {
    if (kb) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = min(kb + u * 512 + lane * 8, K - 8);
#pragma unroll
        for (int r = 0; r < R; r++) wv[u][r] = wload<true>(wr[r] + k);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int kk = kb + u * 512 + lane * 8;
      const bool live = kk < K;
      const int k = min(kk, K - 8);
#pragma unroll
      for (int m = 0; m < MM; m++) {
        bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + (size_t)min(m, M - 1) * xstride + k);
        xv = live ? xv : zero8;
#pragma unroll
        for (int r = 0; r < R; r++) acc[r][m] = dot8(wv[u][r], xv, acc[r][m]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int m = 0; m < MM; m++) acc[r][m] = wave_sum(acc[r][m]);
  epi_dispatch(ep.kind, [&](auto kc) {
    constexpr int EK = decltype(kc)::value;
    if constexpr (EK != EPI_ARGMAX) {
      if (er < R) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
          for (int m = 0; m < MM; m++) v = (lane == r * MM + m) ? acc[r][m] : v;
        const int n = n0 + er;
        if (em < M && n < N) epi_store_pre<bf16, EK>(ep, em, n, v, pre);
      }
    }
  });
}

// Can gemv_rows8 run this shape?  LN: K % 512 == 0 (the gamma / beta pieces), K <= 4096; PLAIN: K % 512 == 0,
// M x K x 2 <= 128 KB.  Not the argmax head.
static bool rows8_ok(bool ln, int M, int K, const Epi& ep) {
  if (M <= 4 || M > 8 || (K % 512) != 0 || ep.kind == EPI_ARGMAX) return false;
  return ln ? K <= 4096 : (size_t)M * K * 2 <= (size_t)128 << 10;
}

template <bool LN>
static void gemv_rows8_launch(const bf16* x, const LnArgs& ln, const bf16* w, int M, int N, int K, const Epi& ep,
                              hipStream_t s) {
  // geometry of the rows kernel: ~ceil(N / 256) rows per block, R rows per wave, 4..16 waves
  const int rows_cu = (N + 255) / 256;
  int R = K <= 2048 ? 2 : 1;
  while ((rows_cu + R - 1) / R > 16 && R < 4) R *= 2;
  const int waves = std::max(4, std::min(16, (rows_cu + R - 1) / R));
  const int cpr = K / 512;
  int U = cpr <= 3 ? cpr : (cpr % 3 == 0 ? 3 : (cpr % 2 == 0 ? 2 : 1));
  while (R * U > 8) U = U % 2 == 0 ? U / 2 : (U == 3 ? 1 : U - 1);  // 4 R U weight VGPRs (1024-thread bound: 128)
  const size_t shm = LN ? (size_t)M * K * 4 + (size_t)K * 4 : (size_t)M * K * 2;
  const int blocks = (N + waves * R - 1) / (waves * R);
  auto go = [&](auto rc, auto uc) {
    constexpr int RR = decltype(rc)::value, UU = decltype(uc)::value;
    static bool attr = false;  // dynamic LDS above 64 KB (bloom-3b / 7b1 widths)
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)gemv_rows8_kernel<RR, UU, LN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      attr = true;
    }
    gemv_rows8_kernel<RR, UU, LN><<<blocks, waves * 64, shm, s>>>(w, x, ln, M, N, K, ep);
  };
  auto gu = [&](auto rc) {
    if (U == 1) go(rc, EpiKindC<1>{});
    else if (U == 2) go(rc, EpiKindC<2>{});
    else if (U == 3) go(rc, EpiKindC<3>{});
    else go(rc, EpiKindC<4>{});
  };
  if (R == 1) gu(EpiKindC<1>{});
  else if (R == 2) gu(EpiKindC<2>{});
  else gu(EpiKindC<4>{});
}


#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill_bf(bf16* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12;
    p[i] = (bf16)(((float)(h >> 8) / 16777216.0f - 0.5f) * scale);
  }
}
__global__ void fill_f(float* p, size_t n, uint32_t seed, float scale, float off) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12;
    p[i] = ((float)(h >> 8) / 16777216.0f - 0.5f) * scale + off;
  }
}

int main() {
  struct Sh { const char* name; int N, K; bool ln; } shapes[] = {
      {"1b1 qkv", 4608, 1536, true}, {"1b1 dense", 1536, 1536, false}, {"1b1 fc1", 6144, 1536, true},
      {"1b1 fc2", 1536, 6144, false}, {"560m qkv", 3072, 1024, true}, {"560m fc2", 1024, 4096, false},
      {"3b qkv", 7680, 2560, true}, {"3b dense", 2560, 2560, false}, {"3b fc1", 10240, 2560, true},
      {"7b1 qkv", 12288, 4096, true}, {"7b1 dense", 4096, 4096, false}, {"7b1 fc1", 16384, 4096, true}};
  const size_t maxw = (size_t)16384 * 4096;
  bf16 *W, *X, *gamma, *beta, *bias, *xn, *out0, *out1; float *x32, *ws; unsigned* tick;
  CK(hipMalloc(&W, maxw * 2)); CK(hipMalloc(&X, 8 * 16384 * 2)); CK(hipMalloc(&x32, 8 * 16384 * 4));
  CK(hipMalloc(&gamma, 16384 * 2)); CK(hipMalloc(&beta, 16384 * 2)); CK(hipMalloc(&bias, 16384 * 2));
  CK(hipMalloc(&xn, 8 * 16384 * 2)); CK(hipMalloc(&out0, 8 * 16384 * 2)); CK(hipMalloc(&out1, 8 * 16384 * 2));
  const size_t cap = (size_t)1024 * 128 * 128;
  CK(hipMalloc(&ws, cap * 4)); CK(hipMalloc(&tick, 4096 * 4)); CK(hipMemset(tick, 0, 4096 * 4));
  fill_bf<<<4096, 256>>>(W, maxw, 1, 0.08f); fill_bf<<<256, 256>>>(X, 8 * 16384, 2, 2.f);
  fill_f<<<256, 256>>>(x32, 8 * 16384, 3, 2.f, 0.3f);
  fill_bf<<<64, 256>>>(gamma, 16384, 4, 0.2f); fill_bf<<<64, 256>>>(beta, 16384, 5, 0.2f); fill_bf<<<64, 256>>>(bias, 16384, 6, 0.05f);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int M : {8, 5}) {
    for (auto& sh : shapes) {
      Epi ep{};
      ep.kind = EPI_GELU; ep.bias = bias; ep.ldo = sh.N;
      ep.sk_ws = ws; ep.sk_tickets = tick; ep.sk_cap = cap; ep.sk_ntickets = 4096;
      LnArgs ln{x32, 1, 0, gamma, beta, 1e-5f};
      float res[2];
      std::vector<bf16> h0((size_t)M * sh.N), h1((size_t)M * sh.N);
      for (int v = 0; v < 2; v++) {
        ep.out_act = v ? out1 : out0;
        auto launch = [&]() {
          if (v == 0) {  // round-4 path
            if (sh.ln) { launch_ln_rows_wave(ln, M, sh.K, xn, 0); gemv_dispatch<false>(xn, LnArgs{}, W, M, sh.N, sh.K, ep, 0); }
            else gemv_dispatch<false>(X, LnArgs{}, W, M, sh.N, sh.K, ep, 0);
          } else if (sh.ln) {
            gemv_rows8_launch<true>(nullptr, ln, W, M, sh.N, sh.K, ep, 0);
          } else {
            gemv_rows8_launch<false>(X, LnArgs{}, W, M, sh.N, sh.K, ep, 0);
          }
        };
        launch();
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int it = 0; it < 7; it++) {
          CK(hipEventRecord(e0));
          for (int rep = 0; rep < 20; rep++) launch();
          CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1));
          t.push_back(ms * 1e3f / 20);
        }
        std::sort(t.begin(), t.end());
        res[v] = t[t.size() / 2];
        CK(hipMemcpy(v ? h1.data() : h0.data(), v ? out1 : out0, (size_t)M * sh.N * 2, hipMemcpyDeviceToHost));
      }
      double md = 0;
      for (size_t i = 0; i < h0.size(); i++) md = std::max(md, (double)fabsf((float)h0[i] - (float)h1[i]));
      const double mb = (double)sh.N * sh.K * 2 / 1e6;
      printf("M=%d %-10s N=%5d K=%5d %s  r4 %7.2f us (%5.0f GB/s)  rows8 %7.2f us (%5.0f GB/s)  max|diff| %.3g\n", M, sh.name,
             sh.N, sh.K, sh.ln ? "LN   " : "plain", res[0], mb / res[0] * 1e3, res[1], mb / res[1] * 1e3, md);
    }
  }
  return 0;
}
