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
                                                       float* __restrict__ lse_out, int V, int ld,
                                                       unsigned int* __restrict__ err) {
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
    long t = targets[row];
  MG_CHECK_INDEX(t, t < V, -1, err, 4u)  // a target >= V would read past the row
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
                                                       bf16_t* __restrict__ dlogits, int V, int ld,
                                                       unsigned int* __restrict__ err) {
  const long row = blockIdx.x;
  long t = targets[row];
  MG_CHECK_INDEX(t, t < V, -1, err, 4u)  // a target >= V would read past the row
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

// ---- one-pass training path (fwd + bwd fused; the row is read from HBM once) ----
// The two-kernel path reads the [M, 50304] bf16 logits twice (fwd: max / sum-exp, bwd: softmax)
// and writes dlogits once: 19.8 GB per B = 64 GPT-2 step.  Here one 1024-thread workgroup holds
// its row in registers (NV 16-B vectors per lane, packed bf16: 4 VGPRs each), reduces max and
// sum-exp over the workgroup, and writes dlogits = (softmax - onehot) / n_valid in the same pass
// (13.2 GB).  grad_out is applied in backward by xent_scale_kernel, which returns at once when it
// is 1 (the training case) -- read on the device, so the step never synchronises with the host.

// out[1] = 1 / n_valid (single block, before the fused pass needs it)
__global__ __launch_bounds__(1024) void xent_count_kernel(const int64_t* __restrict__ targets,
                                                          float* __restrict__ out, int M) {
  __shared__ float red[16];
  float n = 0.f;
  for (int i = threadIdx.x; i < M; i += 1024) n += targets[i] >= 0 ? 1.f : 0.f;
  n = block_sum<16>(n, red);
  if (threadIdx.x == 0) out[1] = n > 0.f ? 1.f / n : 0.f;
}

template <int NV>
__global__ __launch_bounds__(1024) void xent_fused_kernel(const bf16_t* __restrict__ logits,
                                                          const int64_t* __restrict__ targets,
                                                          const float* __restrict__ inv_n,
                                                          float* __restrict__ loss_row,
                                                          bf16_t* __restrict__ dlogits, int V,
                                                          int ld, unsigned int* __restrict__ err) {
  __shared__ float red[32];
  const long row = blockIdx.x;
  const bf16_t* lr = logits + row * ld;
  bf16_t* dr = dlogits + row * ld;
  constexpr uint32_t NEG2 = 0xFF80FF80u;  // two bf16 -inf: columns >= V drop out of max and sum
  uint4 u[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {  // every load issued before any math: NV x 16 B in flight/lane
    const int c = (threadIdx.x + k * 1024) * 8;
    if (c + 8 <= V) {
      u[k] = ld16_nt(lr + c);  // read once
    } else if (c < V) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (c + j < V) ? bf2f(lr[c + j]) : -INFINITY;
      u[k] = pack8(f);
    } else {
      u[k] = make_uint4(NEG2, NEG2, NEG2, NEG2);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float v[8];
    unpack8(u[k], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j]);
  }
  const float gmx = block_max<16>(mx, red);
#pragma unroll
  for (int k = 0; k < NV; ++k) reg_fence(u[k]);  // keep the row packed (4 VGPRs per vector)
  constexpr float L2E = 1.4426950408889634f;
  const float mb = gmx * L2E;
  float sm = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float v[8];
    unpack8(u[k], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) sm += exp2f(fmaf(v[j], L2E, -mb));
  }
  const float gsm = block_sum<16>(sm, red + 16);
#pragma unroll
  for (int k = 0; k < NV; ++k) reg_fence(u[k]);
  const float lse = gmx + __logf(gsm);
  long t = targets[row];
  MG_CHECK_INDEX(t, t < V, -1, err, 4u)  // a target >= V would read past the row
  const float g = (t < 0) ? 0.f : inv_n[0];
  const float lb = lse * L2E;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (threadIdx.x + k * 1024) * 8;
    if (c < ld) {
      float v[8];
      unpack8(u[k], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = g * (exp2f(fmaf(v[j], L2E, -lb)) - ((c + j) == t ? 1.f : 0.f));
      st16_nt(dr + c, pack8(v));  // 6.6 GB at GPT-2 B = 64: bypass L2 / MALL
    }
  }
  if (threadIdx.x == 0) loss_row[row] = (t < 0) ? 0.f : lse - bf2f(lr[t]);
}

// dlogits *= grad_out, skipped on the device when grad_out == 1
__global__ __launch_bounds__(256) void xent_scale_kernel(bf16_t* __restrict__ dl,
                                                         const float* __restrict__ gscale, long n8) {
  const float s = gscale[0];
  if (s == 1.f) return;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    unpack8(ld16(dl + i * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
    st16(dl + i * 8, pack8(v));
  }
}

}  // namespace

namespace mg {

void xent_fwd(const bf16_t* logits, const int64_t* targets, float* loss_row, float* lse, float* out,
              int M, int V, int ld, hipStream_t stream) {
  xent_fwd_kernel<<<M, 256, 0, stream>>>(logits, targets, loss_row, lse, V, ld, debug_err_word());
  xent_finalize_kernel<<<1, 1024, 0, stream>>>(loss_row, targets, out, M);
}

void xent_bwd(const bf16_t* logits, const int64_t* targets, const float* lse, const float* gscale,
              const float* inv_n, bf16_t* dlogits, int M, int V, int ld, hipStream_t stream) {
  xent_bwd_kernel<<<M, 256, 0, stream>>>(logits, targets, lse, gscale, inv_n, dlogits, V, ld, debug_err_word());
}

}  // namespace mg

namespace mg {

int xent_fused_nv(int ld) {  // 16-B vectors per lane of the fused kernel, 0 = not supported
  const int nv = (ld / 8 + 1023) / 1024;
  return (nv >= 4 && nv <= 8) ? nv : 0;
}

void xent_fused(const bf16_t* logits, const int64_t* targets, float* loss_row, float* out,
                bf16_t* dlogits, int M, int V, int ld, hipStream_t stream) {
  xent_count_kernel<<<1, 1024, 0, stream>>>(targets, out, M);
  switch (xent_fused_nv(ld)) {
#define MG_XF(n) \
  case n: xent_fused_kernel<n><<<M, 1024, 0, stream>>>(logits, targets, out + 1, loss_row, dlogits, V, ld, debug_err_word()); break;
    MG_XF(4) MG_XF(5) MG_XF(6) MG_XF(7) MG_XF(8)
#undef MG_XF
    default: break;
  }
  xent_finalize_kernel<<<1, 1024, 0, stream>>>(loss_row, targets, out, M);
}

void xent_scale(bf16_t* dlogits, const float* gscale, long n, hipStream_t stream) {
  const long n8 = n / 8;
  const long blocks = std::min<long>((n8 + 255) / 256, 2048);
  xent_scale_kernel<<<(int)blocks, 256, 0, stream>>>(dlogits, gscale, n8);
}

}  // namespace mg
