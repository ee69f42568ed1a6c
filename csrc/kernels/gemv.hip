// Skinny GEMM ("GEMV") for autoregressive decode on gfx950.
//
// One decode step pushes B <= 8 rows through every projection of the model
// (/root/reference/mingpt/model.py:322-356 re-runs the whole prefix instead; the KV-cache path in
// models/generation.py needs only the new token's rows).  At M = B the MFMA GEMM has 1 row tile:
// 6-24 workgroups walk a K loop one tile at a time and the projection is latency-bound
// (26 us for the 3072 -> 768 MLP projection at B = 1).  The work is a stream of the weight
// matrix (K x N bf16, read once) against B vectors that fit in LDS, so here:
//   * x [B, K] is staged once per workgroup in LDS -- optionally LayerNorm'ed on the way in (the
//     LN that precedes every decode projection but the residual ones; one kernel instead of two);
//   * a wave owns one output column n (outputs <= 8k: every block projection) or 4 (the LM head):
//     its 64 (or 16) lanes read row n = W[n, :] in 16-byte chunks, 4 loads in flight per lane,
//     FMA against the B vectors from LDS;
//   * the lanes of a row fold with xor-shuffles; the row's first lane writes y[b, n] with the same
//     fused epilogues as gemm.hip's forward (bias | bias + GELU | residual + bias), no dropout
//     (inference).
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

constexpr int kGemvMaxB = 8;
constexpr int kGemvMaxK = 4096;  // B x K bf16 of x must fit the LDS staging buffer

template <int B, int LPR>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ x,
                                                   const bf16_t* __restrict__ W,
                                                   bf16_t* __restrict__ y, int N, int K, long ldy,
                                                   const bf16_t* __restrict__ bias,
                                                   const bf16_t* __restrict__ resid, int epi,
                                                   const bf16_t* __restrict__ lnw,
                                                   const bf16_t* __restrict__ lnb, float eps) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [B][K]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int RPW = 64 / LPR;  // rows per wave
  const int g = lane / LPR, j = lane % LPR;
  const int n = (blockIdx.x * 4 + wid) * RPW + g;
  constexpr int STRIDE = LPR * 8;  // elements per load round of a row
  // one row per wave: the whole row (K <= 4096: <= 8 loads per lane) is requested before x is
  // staged and normalised, so the weight stream's memory latency overlaps the LayerNorm's
  constexpr int NPF = LPR == 64 ? kGemvMaxK / STRIDE : 1;
  uint4 wpf[NPF];
  if constexpr (LPR == 64) {
    const bf16_t* wr = W + (long)min(n, N - 1) * K;
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int c = j * 8 + u * STRIDE;
      wpf[u] = c < K ? ld16(wr + c) : make_uint4(0, 0, 0, 0);
    }
  }
  if (lnw) {
    // fused LayerNorm of the B input rows (wave w normalises rows w, w+4): the same lane/chunk
    // order and wave reduction as ln_fwd_kernel, so the staged bf16 rows equal its output
    for (int b = wid; b < B; b += 4) {
      const bf16_t* xr = x + (long)b * K;
      float s = 0.f;
      for (int c = lane * 8; c < K; c += 512) {
        float v[8];
        unpack8(ld16(xr + c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[e];
      }
      const float mu = wave_sum(s) / K;
      float ss = 0.f;
      for (int c = lane * 8; c < K; c += 512) {
        float v[8];
        unpack8(ld16(xr + c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[e] - mu;
          ss += d * d;
        }
      }
      const float rs = rsqrtf(wave_sum(ss) / K + eps);
      for (int c = lane * 8; c < K; c += 512) {
        float v[8], wf[8], bf[8], o[8];
        unpack8(ld16(xr + c), v);
        unpack8(ld16(lnw + c), wf);
        unpack8(ld16(lnb + c), bf);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[e] - mu) * rs * wf[e] + bf[e];
        st16(xs + b * K + c, pack8(o));
      }
    }
  } else {
    for (int i = threadIdx.x * 8; i < B * K; i += 256 * 8) st16(xs + i, ld16(x + i));
  }
  __syncthreads();
  // LPR lanes per output row: 16 (4 rows per wave) for wide outputs (the LM head), 64 (one row per
  // wave, the whole row's loads in flight at once) for the block projections, whose 48-192
  // workgroups at 16 lanes per row left most of the chip idle and the HBM latency exposed
  float acc[B];
#pragma unroll
  for (int b = 0; b < B; ++b) acc[b] = 0.f;
  if constexpr (LPR == 64) {
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int c = j * 8 + u * STRIDE;
      if (c < K) {
        float wf[8];
        unpack8(wpf[u], wf);
#pragma unroll
        for (int b = 0; b < B; ++b) {
          float xf[8];
          unpack8(ld16(xs + b * K + c), xf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[b] = __builtin_fmaf(wf[e], xf[e], acc[b]);
        }
      }
    }
  } else if (n < N) {
    const bf16_t* wr = W + (long)n * K;
    int c = j * 8;
    for (; c + 3 * STRIDE < K; c += 4 * STRIDE) {  // 4 loads in flight per lane
      uint4 wv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) wv[u] = ld16(wr + c + u * STRIDE);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float wf[8];
        unpack8(wv[u], wf);
#pragma unroll
        for (int b = 0; b < B; ++b) {
          float xf[8];
          unpack8(ld16(xs + b * K + c + u * STRIDE), xf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[b] = __builtin_fmaf(wf[e], xf[e], acc[b]);
        }
      }
    }
    for (; c < K; c += STRIDE) {
      float wf[8];
      unpack8(ld16(wr + c), wf);
#pragma unroll
      for (int b = 0; b < B; ++b) {
        float xf[8];
        unpack8(ld16(xs + b * K + c), xf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[b] = __builtin_fmaf(wf[e], xf[e], acc[b]);
      }
    }
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) acc[b] += __shfl_xor(acc[b], o, 64);
  }
  if (n < N && j == 0) {
    const float bv = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      float v = acc[b] + bv;
      if (epi == 2) v = gelu_f(v);
      if (epi == 3) v += bf2f(resid[(long)b * ldy + n]);
      y[(long)b * ldy + n] = f2bf(v);
    }
  }
}

}  // namespace

namespace mg {

bool gemv_supported(int B, int K) { return B >= 1 && B <= kGemvMaxB && K % 8 == 0 && K <= kGemvMaxK; }

void gemv(const bf16_t* x, const bf16_t* W, bf16_t* y, int B, int N, int K, long ldy, const bf16_t* bias,
          const bf16_t* resid, int epi, hipStream_t stream, const bf16_t* lnw, const bf16_t* lnb,
          float eps) {
  const size_t smem = sizeof(bf16_t) * (size_t)B * K;
  // one row per wave (N / 4 workgroups) up to ~8k outputs; 4 rows per wave beyond (the LM head
  // already launches thousands of workgroups and re-stages x in each)
  const bool wide = N > 8192;
  const int grid = wide ? cdiv(N, 16) : cdiv(N, 4);
#define MG_GEMV_CASE(b)                                                                                   \
  case b:                                                                                                 \
    if (wide)                                                                                             \
      gemv_kernel<b, 16><<<grid, 256, smem, stream>>>(x, W, y, N, K, ldy, bias, resid, epi, lnw, lnb, eps); \
    else                                                                                                  \
      gemv_kernel<b, 64><<<grid, 256, smem, stream>>>(x, W, y, N, K, ldy, bias, resid, epi, lnw, lnb, eps); \
    break;
  switch (B) {  // exact row counts: the kernel stages and writes exactly B rows
    MG_GEMV_CASE(1) MG_GEMV_CASE(2) MG_GEMV_CASE(3) MG_GEMV_CASE(4)
    MG_GEMV_CASE(5) MG_GEMV_CASE(6) MG_GEMV_CASE(7) MG_GEMV_CASE(8)
    default: break;
  }
#undef MG_GEMV_CASE
}

}  // namespace mg
