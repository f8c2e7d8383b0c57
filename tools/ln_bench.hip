// tools/ln_bench.hip — the LayerNorm launch of decode and prefill (launch_ln_rows_wave: fp32 rows -> bf16; one wave
// per row until round 6, 4 waves per row above K = 1024 since) against the same math with WPR = 1 / 2 / 4 / 8 waves
// per row (one LDS exchange of the shifted sums), at the batched-decode row counts that keep the LayerNorm launch
// (M = 8..32) and the prefill ones (512, 2048).  Time = median over 5 groups of 200 back-to-back launches between HIP
// events, inputs rotating over 16 row sets.  Outputs compared with the library's (raw bf16 bit distance; large values
// only where a value near zero changes sign).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ln_bench.hip
//        distributed_inference_demo_amd/csrc/attn_prefill.hip -o tools/ln_bench
#include "../distributed_inference_demo_amd/csrc/kernels.hip"
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// WPR waves per row; lane (w, l) holds float4 groups j = i * 64 * WPR + w * 64 + l, i < NV.
template <int NV, int WPR>
__global__ __launch_bounds__(64 * WPR) void ln_rows_multi(LnArgs ln, int K, bf16* __restrict__ out) {
  __shared__ float sh[2 * WPR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* xr = ln.x + (size_t)blockIdx.x * ln.row_stride * K + (size_t)ln.row_offset * K;
  float4 xv[NV];
  uint2 gr[NV], br[NV];
  const float c = xr[0];
#pragma unroll
  for (int i = 0; i < NV; i++) {
    const int k = (i * 64 * WPR + w * 64 + lane) * 4;
    xv[i] = k < K ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    gr[i] = k < K ? *reinterpret_cast<const uint2*>(ln.gamma + k) : make_uint2(0u, 0u);
    br[i] = k < K ? *reinterpret_cast<const uint2*>(ln.beta + k) : make_uint2(0u, 0u);
  }
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    if ((i * 64 * WPR + w * 64 + lane) * 4 < K) {
      const float d0 = xv[i].x - c, d1 = xv[i].y - c, d2 = xv[i].z - c, d3 = xv[i].w - c;
      a1 += (d0 + d1) + (d2 + d3);
      a2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if (WPR > 1) {
    if (lane == 0) { sh[w] = a1; sh[WPR + w] = a2; }
    __syncthreads();
    a1 = 0.f; a2 = 0.f;
#pragma unroll
    for (int j = 0; j < WPR; j++) { a1 += sh[j]; a2 += sh[WPR + j]; }
  }
  const float invk = 1.0f / (float)K;
  const float t1 = a1 * invk, t2 = a2 * invk;
  const float mean = c + t1, rstd = 1.0f / sqrtf(fmaxf(t2 - t1 * t1, 0.f) + ln.eps);
  bf16* orow = out + (size_t)blockIdx.x * K;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    const int k = (i * 64 * WPR + w * 64 + lane) * 4;
    if (k < K) {
      float4 g, b;
      bf16x4_to_f32(gr[i], g);
      bf16x4_to_f32(br[i], b);
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 o;
      o[0] = (bf16)((xv[i].x - mean) * rstd * g.x + b.x);
      o[1] = (bf16)((xv[i].y - mean) * rstd * g.y + b.y);
      o[2] = (bf16)((xv[i].z - mean) * rstd * g.z + b.z);
      o[3] = (bf16)((xv[i].w - mean) * rstd * g.w + b.w);
      *reinterpret_cast<bf16x4*>(orow + k) = o;
    }
  }
}

template <int WPR>
static void launch_multi(const LnArgs& ln, int M, int K, bf16* out) {
  const int nv = (K + 256 * WPR - 1) / (256 * WPR);
  if (nv <= 1) ln_rows_multi<1, WPR><<<M, 64 * WPR>>>(ln, K, out);
  else if (nv <= 2) ln_rows_multi<2, WPR><<<M, 64 * WPR>>>(ln, K, out);
  else if (nv <= 4) ln_rows_multi<4, WPR><<<M, 64 * WPR>>>(ln, K, out);
  else if (nv <= 8) ln_rows_multi<8, WPR><<<M, 64 * WPR>>>(ln, K, out);
  else ln_rows_multi<16, WPR><<<M, 64 * WPR>>>(ln, K, out);
}

int main() {
  const int NSET = 16;
  float* x;
  bf16 *g, *b, *o1, *o2;
  CK(hipMalloc(&x, (size_t)NSET * 2048 * 4096 * 4));
  CK(hipMalloc(&g, 4096 * 2)); CK(hipMalloc(&b, 4096 * 2));
  CK(hipMalloc(&o1, 2048 * 4096 * 2)); CK(hipMalloc(&o2, 2048 * 4096 * 2));
  launch_gen_fill(x, 0, (size_t)NSET * 2048 * 4096, 3, 0, 0);
  launch_gen_fill(g, 1, 4096, 4, 2, 0); launch_gen_fill(b, 1, 4096, 5, 3, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int K : {1536, 2560, 4096}) {
    for (int M : {8, 16, 32, 512, 2048}) {
      auto args = [&](int set) {
        LnArgs ln{};
        ln.x = x + (size_t)set * 2048 * 4096; ln.row_stride = 1; ln.row_offset = 0; ln.gamma = g; ln.beta = b; ln.eps = 1e-5f;
        return ln;
      };
      auto time = [&](const std::function<void(const LnArgs&)>& f) {
        std::vector<float> t;
        for (int i = 0; i < NSET; i++) f(args(i));
        CK(hipDeviceSynchronize());
        for (int rep = 0; rep < 5; rep++) {
          CK(hipEventRecord(e0));
          for (int i = 0; i < 200; i++) f(args(i % NSET));
          CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1));
          t.push_back(ms * 1e3f / 200);
        }
        std::sort(t.begin(), t.end());
        return t[2];
      };
      const float lib = time([&](const LnArgs& ln) { launch_ln_rows_wave(ln, M, K, o1, 0); });
      float tw[4];
      int wi = 0;
      std::vector<uint16_t> h1(M * K), h2(M * K);
      for (int W : {1, 2, 4, 8}) {
        auto f = [&](const LnArgs& ln) {
          if (W == 1) launch_multi<1>(ln, M, K, o2);
          else if (W == 2) launch_multi<2>(ln, M, K, o2);
          else if (W == 4) launch_multi<4>(ln, M, K, o2);
          else launch_multi<8>(ln, M, K, o2);
        };
        tw[wi++] = time(f);
        launch_ln_rows_wave(args(0), M, K, o1, 0);
        f(args(0));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h1.data(), o1, M * K * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), o2, M * K * 2, hipMemcpyDeviceToHost));
        int ulps = 0;
        for (int i = 0; i < M * K; i++) ulps = std::max(ulps, std::abs((int)(int16_t)h1[i] - (int)(int16_t)h2[i]));
        if (ulps > 1) printf("  W=%d: max bf16 ulp difference %d\n", W, ulps);
      }
      printf("K=%5d M=%4d  library %5.2f us | 1 wave/row %5.2f | 2 waves/row %5.2f | 4 waves/row %5.2f | 8 waves/row %5.2f\n",
             K, M, lib, tw[0], tw[1], tw[2], tw[3]);
      fflush(stdout);
    }
  }
  return 0;
}
