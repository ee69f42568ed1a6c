// Token + position embedding (fused gather-add-dropout) for gfx950.
//
// Replaces the reference's GPTEmbedding (/root/reference/mingpt/model.py:193-231): ATen
// embedding gather, broadcast add of the positional table and dropout become one pass.
//
// fwd: out[m, :] = dropout(wte[idx[m], :] + wpe[m % T, :]); one wave per token row, 16-B loads.
// bwd: dwte[idx[m], :] += g[m, :]  -- fp32 atomics into the main-grad buffer, each wave
//      instruction adding 64 contiguous floats (256 contiguous bytes: the full-rate atomic shape);
//      dwpe[t, :] += sum_b g[b*T + t, :]  -- a deterministic column reduction, no atomics.
//      g = dout * dropout-mask (regenerated from the Philox seed).
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ idx,
                                                      const bf16_t* __restrict__ wte,
                                                      const bf16_t* __restrict__ wpe,
                                                      bf16_t* __restrict__ out, int M, int T, int D, int V,
                                                      unsigned int* __restrict__ err,
                                                      uint64_t seed, uint32_t thr, float scale,
                                                      int use_dropout, const uint64_t* sofs,
                                                      const int* __restrict__ pos_dev,
                                                      const unsigned long long* __restrict__ am_part,
                                                      int am_groups, int64_t* __restrict__ tok_out,
                                                      int64_t* __restrict__ seq, long seq_ld) {
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  seed = eff_seed(seed, sofs);
  long tok;
  if (am_part) {
    // greedy decode: this row's token is the argmax the previous step's LM-head GEMV left as one
    // key per workgroup (gemv.hip): a wave max over the keys, first index on ties
    unsigned long long best = 0;
    for (int i = lane; i < am_groups; i += 64) {
      const unsigned long long k = am_part[m * am_groups + i];
      best = k > best ? k : best;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned lo = __shfl_xor((unsigned)best, o, 64), hi = __shfl_xor((unsigned)(best >> 32), o, 64);
      const unsigned long long k = ((unsigned long long)hi << 32) | lo;
      best = k > best ? k : best;
    }
    tok = (long)(0xffffffffu - (uint32_t)best);
    if (lane == 0) {
      if (tok_out) tok_out[m] = tok;
      if (seq) seq[m * seq_ld + *pos_dev] = tok;
    }
  } else {
    tok = idx[m];
  }
  MG_CHECK_INDEX(tok, tok >= 0 && tok < V, 0, err, 1u)
  const int t = pos_dev ? *pos_dev : (int)(m % T);  // decode step: one token at a device position
  for (int c = lane * 8; c < D; c += 512) {
    float a[8], p[8];
    unpack8(ld16(wte + tok * D + c), a);
    unpack8(ld16(wpe + (long)t * D + c), p);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p[j];
    if (use_dropout) rowdrop8(a, seed, m, c, D, thr, scale);
    st16(out + m * D + c, pack8(a));
  }
}

__global__ __launch_bounds__(256) void emb_bwd_wte_kernel(const int64_t* __restrict__ idx,
                                                          const bf16_t* __restrict__ dout,
                                                          float* __restrict__ dwte, int M, int D, int V,
                                                          unsigned int* __restrict__ err,
                                                          uint64_t seed, uint32_t thr, float scale,
                                                          int use_dropout, const uint64_t* sofs) {
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  seed = eff_seed(seed, sofs);
  long tok = idx[m];
  MG_CHECK_INDEX(tok, tok >= 0 && tok < V, 0, err, 2u)
  // 8 columns per lane for the load, then 8 atomic instructions each covering 64 x 4 B contiguous.
  for (int c0 = 0; c0 < D; c0 += 512) {
    const int c = c0 + lane * 8;
    float g[8];
    if (c < D) {
      unpack8(ld16(dout + m * D + c), g);
      if (use_dropout) rowdrop8(g, seed, m, c, D, thr, scale);
    }
    // transpose through lanes so each atomic wave-instruction touches 64 consecutive floats:
    // element j of lane L is column c0 + 8L + j. Atomic k handles columns c0 + 64k + lane,
    // which lives in lane (64k+lane)/8 = 8k + lane/8, element lane%8.
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int src = 8 * k + (lane >> 3);
      float val = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = __shfl(g[j], src, 64);
        if ((lane & 7) == j) val = t;
      }
      const int col = c0 + 64 * k + lane;
      if (col < D) atomicAdd(dwte + tok * D + col, val);
    }
  }
}

// dwpe[t, c] += sum_b g[b*T+t, c]; grid = (T, ceil(D/512)), one wave per (t, 512-col chunk)
__global__ __launch_bounds__(64) void emb_bwd_wpe_kernel(const bf16_t* __restrict__ dout,
                                                         float* __restrict__ dwpe, int B, int T, int D,
                                                         uint64_t seed, uint32_t thr, float scale,
                                                         int use_dropout, const uint64_t* sofs) {
  const int t = blockIdx.x;
  const int c = blockIdx.y * 512 + threadIdx.x * 8;
  if (c >= D) return;
  seed = eff_seed(seed, sofs);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = 0; b < B; ++b) {
    const long m = (long)b * T + t;
    float g[8];
    unpack8(ld16(dout + m * D + c), g);
    if (use_dropout) rowdrop8(g, seed, m, c, D, thr, scale);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += g[j];
  }
  float* dst = dwpe + (long)t * D + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) dst[j] += s[j];
}

}  // namespace

namespace mg {

void embedding_fwd(const int64_t* idx, const bf16_t* wte, const bf16_t* wpe, bf16_t* out, int M,
                   int T, int D, int V, float p, uint64_t seed, hipStream_t stream, const int* pos_dev,
                   const unsigned long long* am_part, int am_groups, int64_t* tok, int64_t* seq,
                   long seq_ld) {
  const uint32_t thr = dropout_threshold16(p);  // the residual-stream mask (common.h)
  emb_fwd_kernel<<<cdiv(M, 4), 256, 0, stream>>>(idx, wte, wpe, out, M, T, D, V, debug_err_word(), seed, thr,
                                                 dropout_scale16(thr), p > 0.f,
                                                 graph_seed_ofs(), pos_dev, am_part, am_groups, tok, seq,
                                                 seq_ld);
}

void embedding_bwd(const int64_t* idx, const bf16_t* dout, float* dwte, float* dwpe, int M, int T,
                   int D, int V, float p, uint64_t seed, hipStream_t stream) {
  const uint32_t thr = dropout_threshold16(p);
  const float scale = dropout_scale16(thr);
  if (dwte)
    emb_bwd_wte_kernel<<<cdiv(M, 4), 256, 0, stream>>>(idx, dout, dwte, M, D, V, debug_err_word(), seed, thr, scale,
                                                       p > 0.f, graph_seed_ofs());
  if (dwpe) {
    dim3 grid(T, cdiv(D, 512));
    emb_bwd_wpe_kernel<<<grid, 64, 0, stream>>>(dout, dwpe, M / T, T, D, seed, thr, scale, p > 0.f,
                                                graph_seed_ofs());
  }
}

unsigned int* debug_err_word() {
#ifdef MG_DEBUG
  static unsigned int* w = nullptr;
  if (!w) {
    (void)hipMalloc(&w, sizeof(unsigned int));
    (void)hipMemset(w, 0, sizeof(unsigned int));
  }
  return w;
#else
  return nullptr;
#endif
}

unsigned int debug_error_bits() {
#ifdef MG_DEBUG
  unsigned int v = 0u;
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(&v, debug_err_word(), sizeof(v), hipMemcpyDeviceToHost);
  (void)hipMemset(debug_err_word(), 0, sizeof(v));
  (void)hipDeviceSynchronize();
  return v;
#else
  return 0u;
#endif
}

}  // namespace mg
