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
//     (inference);
//   * weights are read non-temporally (streamed once per token; MI355X_MICROARCH launches-baseline:
//     nt weight loads ~11 % faster per decode layer);
//   * greedy decode (LM head): the argmax of the logits is fused -- each workgroup publishes its
//     best (value, index) key and the next decode step's embedding kernel reduces them into the
//     token (and advances the device position), so a captured decode step can be replayed back
//     to back with no host round trip per token.
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

constexpr int kGemvMaxB = 8;
constexpr int kGemvMaxK = 4096;  // B x K bf16 of x must fit the LDS staging buffer

// order-preserving key of a float (larger float -> larger key), index in the low half inverted
// so that the max key is the FIRST index among equal values (torch.argmax)
MG_DEVICE unsigned long long amax_key(float v, int n) {
  const uint32_t u = __float_as_uint(v);
  const uint32_t k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)k << 32) | (uint32_t)(0xffffffffu - (uint32_t)n);
}
MG_DEVICE unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }

// Fused greedy argmax, first half: every workgroup publishes its best (value, index) key per row
// to part[b][workgroup] with plain stores, and workgroup 0 advances the device position.  The
// cross-workgroup reduction is the NEXT kernel's (the decode step's embedding kernel, at a launch
// boundary: no atomics, no hand-off).  A last-arrival reduction inside this kernel cost ~5 us per
// token (store drain + returning atomics on counters; MI355X_MICROARCH 'dequeue').
template <int B>
MG_DEVICE void gemv_argmax(const GemvArgmax& am, const unsigned long long (&key)[B], bool mine, int row) {
  __shared__ unsigned long long kk[B][16];
  if (mine) {  // this lane's best over the rows it produced (0: none)
#pragma unroll
    for (int b = 0; b < B; ++b) kk[b][row] = key[b];
  }
  __syncthreads();
  if (threadIdx.x < B) {
    unsigned long long best = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) best = umax64(best, kk[threadIdx.x][r]);
    am.part[(long)threadIdx.x * gridDim.x + blockIdx.x] = best;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *am.pos += 1;  // nothing else in this kernel reads it
}

template <int B, int LPR, bool NTW>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ x,
                                                   const bf16_t* __restrict__ W,
                                                   bf16_t* __restrict__ y, int N, int K, long ldy,
                                                   const bf16_t* __restrict__ bias,
                                                   const bf16_t* __restrict__ resid, int epi,
                                                   const bf16_t* __restrict__ lnw,
                                                   const bf16_t* __restrict__ lnb, float eps,
                                                   const GemvArgmax am) {
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
      wpf[u] = c < K ? (NTW ? ld16_nt(wr + c) : ld16(wr + c)) : make_uint4(0, 0, 0, 0);
    }
  }
  if (lnw) {
    // fused LayerNorm of the B input rows (wave w normalises rows w, w+4): the same lane/chunk
    // order and wave reduction as ln_fwd_kernel, so the staged bf16 rows equal its output
    // K <= 1024 (GPT-2 small / medium): the row, gamma and beta chunks are loaded once into
    // registers (one memory round trip instead of three dependent L2 reads); wider rows re-read
    if (K <= 1024) {
      for (int b = wid; b < B; b += 4) {
        const bf16_t* xr = x + (long)b * K;
        uint4 xv[2], wv[2], bv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = lane * 8 + u * 512;
          const bool ok = c < K;
          xv[u] = ok ? ld16(xr + c) : make_uint4(0, 0, 0, 0);
          wv[u] = ok ? ld16(lnw + c) : make_uint4(0, 0, 0, 0);
          bv[u] = ok ? ld16(lnb + c) : make_uint4(0, 0, 0, 0);
        }
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float v[8];
          unpack8(xv[u], v);
#pragma unroll
          for (int e = 0; e < 8; ++e) s += v[e];  // zero chunks past K add nothing
        }
        const float mu = wave_sum(s) / K;
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (lane * 8 + u * 512 < K) {
            float v[8];
            unpack8(xv[u], v);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = v[e] - mu;
              ss += d * d;
            }
          }
        }
        const float rs = rsqrtf(wave_sum(ss) / K + eps);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = lane * 8 + u * 512;
          if (c < K) {
            float v[8], wf[8], bf[8], o[8];
            unpack8(xv[u], v);
            unpack8(wv[u], wf);
            unpack8(bv[u], bf);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (v[e] - mu) * rs * wf[e] + bf[e];
            st16(xs + b * K + c, pack8(o));
          }
        }
      }
    } else {
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
    }
  } else {
    for (int i = threadIdx.x * 8; i < B * K; i += 256 * 8) st16(xs + i, ld16(x + i));
  }
  __syncthreads();
  // LPR lanes per output row: 16 (4 rows per wave) for wide outputs (the LM head), 64 (one row per
  // wave, the whole row's loads in flight at once) for the block projections, whose 48-192
  // workgroups at 16 lanes per row left most of the chip idle and the HBM latency exposed
  auto epilogue = [&](float (&acc)[B], int n) {
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
        const bf16_t o = f2bf(v);
        y[(long)b * ldy + n] = o;
        acc[b] = bf2f(o);  // the argmax ranks the stored (bf16) logits
      }
    }
  };
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
    epilogue(acc, n);
  } else {
    // wide outputs: grid-stride over 16-row blocks (a few hundred workgroups stage x once each;
    // the fused argmax then pays its cross-workgroup hand-off once per workgroup)
    unsigned long long best[B];
#pragma unroll
    for (int b = 0; b < B; ++b) best[b] = 0ull;
    // work items = (16-row block, 1024-column segment); the next item's 8 chunks per lane are
    // requested before the current item's FMAs, so every lane keeps a full item in flight
    const int nrb = (N + 15) / 16;
    const int nseg = (K + 16 * 8 * 8 - 1) / (16 * 8 * 8);
    const int nit = (blockIdx.x < nrb ? (nrb - 1 - blockIdx.x) / gridDim.x + 1 : 0) * nseg;
    auto load_item = [&](int it, uint4 (&r)[8]) {
      const int rb = blockIdx.x + (it / nseg) * gridDim.x, seg = it % nseg;
      const int nr = min((rb * 4 + wid) * RPW + g, N - 1);
      const bf16_t* wr = W + (long)nr * K + seg * 1024;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = seg * 1024 + j * 8 + u * STRIDE;
        r[u] = c < K ? (NTW ? ld16_nt(wr + j * 8 + u * STRIDE) : ld16(wr + j * 8 + u * STRIDE))
                     : make_uint4(0, 0, 0, 0);
      }
    };
    uint4 cur[8], nxt[8];
    if (nit > 0) load_item(0, cur);
    for (int it = 0; it < nit; ++it) {
      if (it + 1 < nit) load_item(it + 1, nxt);
      const int rb = blockIdx.x + (it / nseg) * gridDim.x, seg = it % nseg;
      const int nr = (rb * 4 + wid) * RPW + g;
      if (seg == 0) {
#pragma unroll
        for (int b = 0; b < B; ++b) acc[b] = 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = seg * 1024 + j * 8 + u * STRIDE;
        if (c < K) {
          float wf[8];
          unpack8(cur[u], wf);
#pragma unroll
          for (int b = 0; b < B; ++b) {
            float xf[8];
            unpack8(ld16(xs + b * K + c), xf);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[b] = __builtin_fmaf(wf[e], xf[e], acc[b]);
          }
        }
      }
      if (seg == nseg - 1) {
        epilogue(acc, nr);
        if (am.part && nr < N && j == 0) {
#pragma unroll
          for (int b = 0; b < B; ++b) best[b] = umax64(best[b], amax_key(acc[b], nr));
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) cur[u] = nxt[u];
    }
    if (am.part) gemv_argmax<B>(am, best, j == 0, wid * RPW + g);
  }
}

}  // namespace

namespace mg {

bool gemv_supported(int B, int K) { return B >= 1 && B <= kGemvMaxB && K % 8 == 0 && K <= kGemvMaxK; }

// wide outputs: a few workgroups per CU, grid-striding over the 16-row blocks
int gemv_wide_cap() {
  static int cap = 0;
  if (!cap) {
    const char* e = getenv("MINGPT_GEMV_WIDE_GRID");
    cap = e ? atoi(e) : 512;
    if (cap <= 0) cap = 512;
  }
  return cap;
}
// (B <= 2: twice the workgroups -- the LM head's 16-row blocks are then latency-, not
// bandwidth-bound: 3,359 / 3,335 vs 3,319 / 3,302 tok/s at B = 1, equal at B = 8;
// profiles/round2_s8_decode_gemv_policy_ab.jsonl)
int gemv_grid(int N, int B) {
  if (N <= 8192) return cdiv(N, 4);
  const char* e = getenv("MINGPT_GEMV_WIDE_GRID");
  return min(cdiv(N, 16), (e || B > 2) ? gemv_wide_cap() : 1024);
}
// weight loads non-temporal (default) or default cache policy (MINGPT_GEMV_NT=0): the decode step
// re-reads the same ~250 MB of GPT-2 weights every token, about the Infinity Cache's size
bool gemv_nt_weights() {
  static int nt = -1;
  if (nt < 0) {
    const char* e = getenv("MINGPT_GEMV_NT");
    nt = e ? atoi(e) != 0 : 1;
  }
  return nt != 0;
}
// argmax partials: one 8-byte key per (row, workgroup)

void gemv(const bf16_t* x, const bf16_t* W, bf16_t* y, int B, int N, int K, long ldy, const bf16_t* bias,
          const bf16_t* resid, int epi, hipStream_t stream, const bf16_t* lnw, const bf16_t* lnb,
          float eps, const GemvArgmax* am) {
  const size_t smem = sizeof(bf16_t) * (size_t)B * K;
  // one row per wave (N / 4 workgroups) up to ~8k outputs; 4 rows per wave beyond (the LM head
  // already launches thousands of workgroups and re-stages x in each)
  const bool wide = N > 8192;
  const int grid = gemv_grid(N, B);
  const GemvArgmax amv = am ? *am : GemvArgmax{nullptr, nullptr};
  const bool ntw = gemv_nt_weights();
#define MG_GEMV_LAUNCH(b, lpr)                                                                                        \
  if (ntw) gemv_kernel<b, lpr, true><<<grid, 256, smem, stream>>>(x, W, y, N, K, ldy, bias, resid, epi, lnw, lnb, eps, amv); \
  else gemv_kernel<b, lpr, false><<<grid, 256, smem, stream>>>(x, W, y, N, K, ldy, bias, resid, epi, lnw, lnb, eps, amv);
#define MG_GEMV_CASE(b)        \
  case b:                      \
    if (wide) {                \
      MG_GEMV_LAUNCH(b, 16)    \
    } else {                   \
      MG_GEMV_LAUNCH(b, 64)    \
    }                          \
    break;
  switch (B) {  // exact row counts: the kernel stages and writes exactly B rows
    MG_GEMV_CASE(1) MG_GEMV_CASE(2) MG_GEMV_CASE(3) MG_GEMV_CASE(4)
    MG_GEMV_CASE(5) MG_GEMV_CASE(6) MG_GEMV_CASE(7) MG_GEMV_CASE(8)
    default: break;
  }
#undef MG_GEMV_CASE
#undef MG_GEMV_LAUNCH
}

}  // namespace mg
