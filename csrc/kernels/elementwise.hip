// Elementwise epilogue kernels (gfx950), used where an epilogue is not fused into a GEMM,
// plus the bias-gradient column reduction.
//
//   bias_act_fwd:      y = act(x + b)             act in {identity, gelu}; optionally keeps pre
//   bias_drop_resid:   y = r + dropout(x + b)     (attn c_proj / mlp c_proj residual epilogue)
//   gelu_bwd:          dx = dy * gelu'(pre)
//   dropout_bwd:       dx = dy * mask * scale     (mask regenerated from the Philox seed; common.h rowdrop)
//   bias_grad:         db[n] += sum_m dy[m, n]    (fp32 accumulate into the main grad)
//
// All tensors are [M, N] bf16 row-major with N % 8 == 0; 8 elements (16 B) per lane.
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

constexpr int kGrid = 4096;

__global__ __launch_bounds__(256) void bias_act_kernel(const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ pre,
                                                       bf16_t* __restrict__ y, long n8, int N,
                                                       int act) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    const int c = (int)(e % N);
    float v[8], bb[8];
    unpack8(ld16(x + e), v);
    if (b) {
      unpack8(ld16(b + c), bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bb[j];
    }
    if (act == 1) {
      if (pre) st16(pre + e, pack8(v));
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j]);
    }
    st16(y + e, pack8(v));
  }
}

__global__ __launch_bounds__(256) void bias_drop_resid_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ b, const bf16_t* __restrict__ r,
    bf16_t* __restrict__ y, long n8, int N, uint64_t seed, uint32_t thr, float scale, int use_drop) {
  const uint32_t n8row = (uint32_t)(N >> 3);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    const long m = (long)((uint64_t)i / n8row);
    const int c = (int)(e - m * N);
    float v[8], bb[8], rr[8];
    unpack8(ld16(x + e), v);
    if (b) {
      unpack8(ld16(b + c), bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bb[j];
    }
    if (use_drop) rowdrop8(v, seed, m, c, N, thr, scale);
    unpack8(ld16(r + e), rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += rr[j];
    st16(y + e, pack8(v));
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ pre,
                                                       bf16_t* __restrict__ dx, long n8) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    float g[8], p[8];
    unpack8(ld16(dy + e), g);
    unpack8(ld16(pre + e), p);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= gelu_grad(p[j]);
    st16(dx + e, pack8(g));
  }
}

__global__ __launch_bounds__(256) void dropout_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          bf16_t* __restrict__ dx, long n8, int N,
                                                          uint64_t seed, uint32_t thr, float scale) {
  const uint32_t n8row = (uint32_t)(N >> 3);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    const long m = (long)((uint64_t)i / n8row);
    float g[8];
    unpack8(ld16(dy + e), g);
    rowdrop8(g, seed, m, (int)(e - m * N), N, thr, scale);
    st16(dx + e, pack8(g));
  }
}

// Same row/column decomposition as bias_grad_kernel below, fused with the residual-dropout
// backward: dx = dy * mask / (1-p) is written and its column sums are accumulated in one pass.
__global__ __launch_bounds__(256) void dropout_bias_grad_kernel(const bf16_t* __restrict__ dy,
                                                                bf16_t* __restrict__ dx,
                                                                float* __restrict__ db, int M, int N,
                                                                uint64_t seed, uint32_t thr,
                                                                float scale) {
  __shared__ __attribute__((aligned(16))) float red[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + lane * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (long r = (long)blockIdx.y * 4 + w; r < M; r += (long)gridDim.y * 4) {
      float g[8];
      const long e = r * N + c;
      unpack8(ld16(dy + e), g);
      rowdrop8(g, seed, r, c, N, thr, scale);
      st16(dx + e, pack8(g));
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += g[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = s[j];
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int col = blockIdx.x * 512 + k;
    if (col < N) atomicAdd(db + col, red[0][k] + red[1][k] + red[2][k] + red[3][k]);
  }
}

// grid = (ceil(N/512), RB); block = 256 (4 waves).  Wave w of block (cx, ry) sums rows
// r = ry*4 + w, stepping by 4*RB, over columns cx*512 + lane*8 .. +8; LDS folds the 4 waves;
// one fp32 atomic per column per block-row (RB-way, tiny).
__global__ __launch_bounds__(256) void bias_grad_kernel(const bf16_t* __restrict__ dy,
                                                        float* __restrict__ db, int M, int N) {
  __shared__ __attribute__((aligned(16))) float red[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + lane * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (long r = (long)blockIdx.y * 4 + w; r < M; r += (long)gridDim.y * 4) {
      float g[8];
      unpack8(ld16(dy + r * N + c), g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += g[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = s[j];
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int col = blockIdx.x * 512 + k;
    if (col < N) atomicAdd(db + col, red[0][k] + red[1][k] + red[2][k] + red[3][k]);
  }
}

int grid_for(long n8) { return (int)std::min<long>(kGrid, (n8 + 255) / 256); }

}  // namespace

namespace mg {

void bias_act_fwd(const bf16_t* x, const bf16_t* b, bf16_t* pre, bf16_t* y, long M, int N, int act,
                  hipStream_t stream) {
  const long n8 = M * N / 8;
  bias_act_kernel<<<grid_for(n8), 256, 0, stream>>>(x, b, pre, y, n8, N, act);
}

void bias_dropout_residual(const bf16_t* x, const bf16_t* b, const bf16_t* r, bf16_t* y, long M,
                           int N, float p, uint64_t seed, hipStream_t stream) {
  const long n8 = M * N / 8;
  const uint32_t thr = dropout_threshold8(p);
  bias_drop_resid_kernel<<<grid_for(n8), 256, 0, stream>>>(x, b, r, y, n8, N, seed, thr,
                                                           dropout_scale8(thr), thr > 0);
}

void gelu_bwd(const bf16_t* dy, const bf16_t* pre, bf16_t* dx, long n, hipStream_t stream) {
  gelu_bwd_kernel<<<grid_for(n / 8), 256, 0, stream>>>(dy, pre, dx, n / 8);
}

void dropout_bwd(const bf16_t* dy, bf16_t* dx, long M, int N, float p, uint64_t seed,
                 hipStream_t stream) {
  const uint32_t thr = dropout_threshold8(p);
  const long n8 = M * N / 8;
  dropout_bwd_kernel<<<grid_for(n8), 256, 0, stream>>>(dy, dx, n8, N, seed, thr, dropout_scale8(thr));
}

void dropout_bias_grad(const bf16_t* dy, bf16_t* dx, float* db, long M, int N, float p, uint64_t seed,
                       hipStream_t stream) {
  const int cx = cdiv(N, 512);
  int ry = (int)std::min<long>(512, (M + 3) / 4);
  while (cx * ry > 2048 && ry > 1) ry >>= 1;
  const uint32_t thr = dropout_threshold8(p);
  dropout_bias_grad_kernel<<<dim3(cx, ry), 256, 0, stream>>>(dy, dx, db, (int)M, N, seed, thr,
                                                             dropout_scale8(thr));
}

void bias_grad(const bf16_t* dy, float* db, long M, int N, hipStream_t stream) {
  const int cx = cdiv(N, 512);
  int ry = (int)std::min<long>(512, (M + 3) / 4);
  while (cx * ry > 2048 && ry > 1) ry >>= 1;  // ~2048 blocks: every CU busy, few atomics per column
  bias_grad_kernel<<<dim3(cx, ry), 256, 0, stream>>>(dy, db, (int)M, N);
}

}  // namespace mg
