// attn_merge.h — split-context decode attention: the consumer merges the partials.
//
// Decode attention may split each (row, head)'s context over `nsplit` blocks; each leaves a partial
// (running max m, sum l, unnormalised context acc[hd]) in the AttnParts workspace.  The kernel that
// consumes ctx — the dense GEMV, which loads the whole ctx row anyway — combines the partials of
// every head in its prologue: no ticket, no merge kernel, no extra round trip on the critical path.
//   ctx[b][head*hd + d] = bf16( sum_s exp(m_s - M) acc_s[d] / sum_s exp(m_s - M) l_s ),  M = max_s m_s
// (flash-decoding combine of the fp32 softmax of modeling_bloom.py:283; the bf16 rounding is the
// one attn_decode_kernel applies when it writes ctx itself).
#pragma once
#include "common.h"
#include "kernels.h"

constexpr int kPartsMaxSplit = 4;  // splits a consumer merges (attention_decode_splits caps to it)

struct PartsRegs {
  float m[kPartsMaxSplit], l[kPartsMaxSplit];
  float4 a[kPartsMaxSplit];
};

// Context columns [e, e+4) of row b (e % 4 == 0, head_dim % 4 == 0): issue the loads of every
// split's (m, l) and acc[d..d+3].  LD1(ptr, element) -> float, LD4(ptr, element) -> float4.
template <typename LD1, typename LD4>
__device__ __forceinline__ void attn_parts_load(const AttnParts& p, int b, int e, LD1 ld1, LD4 ld4, PartsRegs& r) {
  const int head = e / p.head_dim, d = e - head * p.head_dim;
  const size_t pair = (size_t)(p.slot + b) * p.n_head + head;
  const size_t ab = pair * p.max_chunks * p.head_dim + d;
  const size_t mb = pair * p.max_chunks * 2;
#pragma unroll
  for (int s = 0; s < kPartsMaxSplit; s++) {
    const int t = min(s, p.nsplit - 1);  // unused slots re-read the last split (masked below)
    r.m[s] = ld1(p.ml, mb + 2 * t);
    r.l[s] = ld1(p.ml, mb + 2 * t + 1);
    r.a[s] = ld4(p.acc, ab + (size_t)t * p.head_dim);
  }
}

__device__ __forceinline__ void attn_parts_combine(int nsplit, const PartsRegs& r, float out[4]) {
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < kPartsMaxSplit; s++)
    if (s < nsplit) M = fmaxf(M, r.m[s]);
  float L = 0.f, o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
  for (int s = 0; s < kPartsMaxSplit; s++) {
    if (s < nsplit && r.m[s] != -INFINITY) {  // a split past the context end holds nothing
      const float w = __expf(r.m[s] - M);
      L += w * r.l[s];
      o0 += w * r.a[s].x; o1 += w * r.a[s].y; o2 += w * r.a[s].z; o3 += w * r.a[s].w;
    }
  }
  out[0] = o0 / L; out[1] = o1 / L; out[2] = o2 / L; out[3] = o3 / L;
}
