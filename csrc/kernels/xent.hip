// Fused softmax cross-entropy for gfx950 (replaces ATen log_softmax + nll_loss and their
// backwards; reference /root/reference/mingpt/model.py:316-318, ignore_index=-1).
//
// logits: [M, ld] bf16 with V <= ld valid columns (ld is padded to a multiple of 8 so every
// row is 16-B aligned; the pad columns are never read in fwd and are written as 0 in bwd).
//
// fwd: one 256-thread block per row, single pass with an online (max, sum-exp) per lane, one
//      block reduction, loss_row = lse - logit[target] (0 for ignored rows), lse saved.
//      A finalize kernel sums the rows and counts the valid targets into {loss, 1/n_valid}
//      on the device: no host synchronisation anywhere in the loss.
// bwd: dlogits = (softmax - onehot) * grad_out / n_valid; grad_out and 1/n_valid are read from
//      device memory, so the whole step stays asynchronous (and graph-capturable).
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

__global__ __launch_bounds__(256) void xent_fwd_kernel(const bf16_t* __restrict__ logits,
                                                       const int64_t* __restrict__ targets,
                                                       float* __restrict__ loss_row,
                                                       float* __restrict__ lse_out, int V, int ld) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const bf16_t* lr = logits + row * ld;
  float mx = -INFINITY, sm = 0.f;
  const int V8 = V & ~7;
  for (int c = threadIdx.x * 8; c < V8; c += 256 * 8) {
    float v[8];
    unpack8(ld16(lr + c), v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    if (lm > mx) {
      sm *= __expf(mx - lm);
      mx = lm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sm += __expf(v[j] - mx);
  }
  for (int c = V8 + threadIdx.x; c < V; c += 256) {  // tail (V % 8)
    const float v = bf2f(lr[c]);
    if (v > mx) {
      sm *= __expf(mx - v);
      mx = v;
    }
    sm += __expf(v - mx);
  }
  const float gmx = block_max<4>(mx, red);
  sm = (mx == -INFINITY) ? 0.f : sm * __expf(mx - gmx);
  const float gsm = block_sum<4>(sm, red + 4);
  if (threadIdx.x == 0) {
    const float lse = gmx + __logf(gsm);
    lse_out[row] = lse;
    const long t = targets[row];
    loss_row[row] = (t < 0) ? 0.f : lse - bf2f(lr[t]);
  }
}

// out[0] = sum(loss_row) / n_valid ; out[1] = 1 / n_valid  (single block)
__global__ __launch_bounds__(1024) void xent_finalize_kernel(const float* __restrict__ loss_row,
                                                             const int64_t* __restrict__ targets,
                                                             float* __restrict__ out, int M) {
  __shared__ float red[32];
  float s = 0.f, n = 0.f;
  for (int i = threadIdx.x; i < M; i += 1024) {
    s += loss_row[i];
    n += targets[i] >= 0 ? 1.f : 0.f;
  }
  s = block_sum<16>(s, red);
  n = block_sum<16>(n, red + 16);
  if (threadIdx.x == 0) {
    const float inv = n > 0.f ? 1.f / n : 0.f;
    out[0] = s * inv;
    out[1] = inv;
  }
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const bf16_t* __restrict__ logits,
                                                       const int64_t* __restrict__ targets,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ gscale,
                                                       const float* __restrict__ inv_n,
                                                       bf16_t* __restrict__ dlogits, int V, int ld) {
  const long row = blockIdx.x;
  const long t = targets[row];
  const float g = (t < 0) ? 0.f : gscale[0] * inv_n[0];
  const float l = lse[row];
  const bf16_t* lr = logits + row * ld;
  bf16_t* dr = dlogits + row * ld;
  for (int c = threadIdx.x * 8; c < ld; c += 256 * 8) {
    float v[8];
    if (c + 8 <= V) {
      unpack8(ld16(lr + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = g * (__expf(v[j] - l) - ((c + j) == t ? 1.f : 0.f));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cj = c + j;
        v[j] = cj < V ? g * (__expf(bf2f(lr[cj]) - l) - (cj == t ? 1.f : 0.f)) : 0.f;
      }
    }
    st16(dr + c, pack8(v));
  }
}

}  // namespace

namespace mg {

void xent_fwd(const bf16_t* logits, const int64_t* targets, float* loss_row, float* lse, float* out,
              int M, int V, int ld, hipStream_t stream) {
  xent_fwd_kernel<<<M, 256, 0, stream>>>(logits, targets, loss_row, lse, V, ld);
  xent_finalize_kernel<<<1, 1024, 0, stream>>>(loss_row, targets, out, M);
}

void xent_bwd(const bf16_t* logits, const int64_t* targets, const float* lse, const float* gscale,
              const float* inv_n, bf16_t* dlogits, int M, int V, int ld, hipStream_t stream) {
  xent_bwd_kernel<<<M, 256, 0, stream>>>(logits, targets, lse, gscale, inv_n, dlogits, V, ld);
}

}  // namespace mg
