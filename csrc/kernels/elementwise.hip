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
    bf16_t* __restrict__ y, long n8, int N, uint64_t seed, uint32_t thr, float scale, int use_drop,
    const uint64_t* sofs) {
  const uint32_t n8row = (uint32_t)(N >> 3);
  seed = eff_seed(seed, sofs);
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
                                                          uint64_t seed, uint32_t thr, float scale,
                                                          const uint64_t* sofs) {
  const uint32_t n8row = (uint32_t)(N >> 3);
  seed = eff_seed(seed, sofs);
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
template <int CVB>
__global__ __launch_bounds__(256) void dropout_bias_grad_kernel(const bf16_t* __restrict__ dy,
                                                                bf16_t* __restrict__ dx,
                                                                float* __restrict__ db, int M, int N,
                                                                uint64_t seed, uint32_t thr,
                                                                float scale, const uint64_t* sofs) {
  constexpr int RG = 256 / CVB;  // rows in flight per block
  __shared__ __attribute__((aligned(16))) float red[RG][CVB * 8];
  seed = eff_seed(seed, sofs);
  const int cv = threadIdx.x % CVB, rg = threadIdx.x / CVB;
  const int c = (blockIdx.x * CVB + cv) * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (long r = (long)blockIdx.y * RG + rg; r < M; r += (long)gridDim.y * RG) {
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
  for (int j = 0; j < 8; ++j) red[rg][cv * 8 + j] = s[j];
  __syncthreads();
  for (int k = threadIdx.x; k < CVB * 8; k += 256) {
    const int col = blockIdx.x * CVB * 8 + k;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RG; ++i) t += red[i][k];
    if (col < N) atomicAdd(db + col, t);
  }
}

// grid = (ceil(N / (8 CVB)), RB); block = 256 threads = RG = 256 / CVB row groups of CVB lanes,
// each lane owning 8 columns.  CVB = 32 when N / 8 is a multiple of 32 but not of 64 (N = 768:
// three full blocks instead of two with a quarter of the lanes idle).  Row group g of block
// (cx, ry) sums rows r = ry*RG + g, stepping by RG*RB; LDS folds the row groups; one fp32 atomic
// per column per block-row (RB-way, tiny).
template <int CVB>
__global__ __launch_bounds__(256) void bias_grad_kernel(const bf16_t* __restrict__ dy,
                                                        float* __restrict__ db, int M, int N, long ld) {
  constexpr int RG = 256 / CVB;
  __shared__ __attribute__((aligned(16))) float red[RG][CVB * 8];
  const int cv = threadIdx.x % CVB, rg = threadIdx.x / CVB;
  const int c = (blockIdx.x * CVB + cv) * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (long r = (long)blockIdx.y * RG + rg; r < M; r += (long)gridDim.y * RG) {
      float g[8];
      unpack8(ld16(dy + r * ld + c), g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += g[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cv * 8 + j] = s[j];
  __syncthreads();
  for (int k = threadIdx.x; k < CVB * 8; k += 256) {
    const int col = blockIdx.x * CVB * 8 + k;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RG; ++i) t += red[i][k];
    if (col < N) atomicAdd(db + col, t);
  }
}

// dst[c][r] = src[r][c] for a [R, C] bf16 matrix; dst rows have ldd >= R elements, the columns
// R..ldd-1 are zero-filled (padded-K operands).  128x128 tiles, 256 threads: thread (rb, cb) loads
// the 8x8 block at rows 8rb.., cols 8cb.. with 16-byte loads (16 threads = 256 contiguous bytes of a
// row), transposes it in registers (one v_perm_b32 per output dword), and swaps blocks through
// LDS (16-byte units, XOR-swizzled) so the stores are 16 threads x 16 B of one output row.
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ src,
                                                        bf16_t* __restrict__ dst, int R, int C,
                                                        int ldd) {
  __shared__ uint4 t[16 * 8 * 16];  // [cb][k][rb ^ cb]
  const int r0 = blockIdx.y * 128, c0 = blockIdx.x * 128;
  {
    const int rb = threadIdx.x >> 4, cb = threadIdx.x & 15;
    uint32_t w[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = r0 + 8 * rb + i, c = c0 + 8 * cb;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < R) {
        if (c + 8 <= C) {
          v = ld16(src + (long)r * C + c);
        } else if (c < C) {
          alignas(16) bf16_t e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          for (int q = 0; q < 8 && c + q < C; ++q) e[q] = src[(long)r * C + c + q];
          v = *reinterpret_cast<const uint4*>(e);
        }
      }
      w[i][0] = v.x; w[i][1] = v.y; w[i][2] = v.z; w[i][3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // output row k of the block = input column k
      uint32_t o[4];
#pragma unroll
      for (int d = 0; d < 4; ++d)
        o[d] = __builtin_amdgcn_perm(w[2 * d + 1][k >> 1], w[2 * d][k >> 1], (k & 1) ? 0x07060302u : 0x05040100u);
      t[(cb * 8 + k) * 16 + (rb ^ cb)] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  __syncthreads();
  const int cb = threadIdx.x >> 4, rb = threadIdx.x & 15;
  const int r = r0 + 8 * rb;
  if (r >= ldd) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + 8 * cb + k;
    if (c >= C) break;
    const uint4 v = t[(cb * 8 + k) * 16 + (rb ^ cb)];
    if (r + 8 <= ldd) {
      st16(dst + (long)c * ldd + r, v);
    } else {
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
      for (int q = 0; r + q < ldd; ++q) dst[(long)c * ldd + r + q] = e[q];
    }
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
  const uint32_t thr = dropout_threshold16(p);
  bias_drop_resid_kernel<<<grid_for(n8), 256, 0, stream>>>(x, b, r, y, n8, N, seed, thr,
                                                           dropout_scale16(thr), thr > 0,
                                                           graph_seed_ofs());
}

void gelu_bwd(const bf16_t* dy, const bf16_t* pre, bf16_t* dx, long n, hipStream_t stream) {
  gelu_bwd_kernel<<<grid_for(n / 8), 256, 0, stream>>>(dy, pre, dx, n / 8);
}

void dropout_bwd(const bf16_t* dy, bf16_t* dx, long M, int N, float p, uint64_t seed,
                 hipStream_t stream) {
  const uint32_t thr = dropout_threshold16(p);
  const long n8 = M * N / 8;
  dropout_bwd_kernel<<<grid_for(n8), 256, 0, stream>>>(dy, dx, n8, N, seed, thr, dropout_scale16(thr),
                                                       graph_seed_ofs());
}

// lanes per row chunk: 32 when it fills every lane and 64 would not
static int bias_cvb(int N) { return ((N / 8) % 64 != 0 && (N / 8) % 32 == 0) ? 32 : 64; }

static dim3 bias_grid(long M, int N, int cvb) {
  const int cx = cdiv(N, cvb * 8);
  int ry = (int)std::max<long>(1, std::min<long>(512, M / 64));  // >= 64 rows per block: few atomics
  while (cx * ry > 2048 && ry > 1) ry >>= 1;  // ~2048 blocks: every CU busy, few atomics per column
  return dim3(cx, ry);
}

void dropout_bias_grad(const bf16_t* dy, bf16_t* dx, float* db, long M, int N, float p, uint64_t seed,
                       hipStream_t stream) {
  const uint32_t thr = dropout_threshold16(p);
  const int cvb = bias_cvb(N);
  const dim3 grid = bias_grid(M, N, cvb);
  if (cvb == 32)
    dropout_bias_grad_kernel<32><<<grid, 256, 0, stream>>>(dy, dx, db, (int)M, N, seed, thr,
                                                           dropout_scale16(thr), graph_seed_ofs());
  else
    dropout_bias_grad_kernel<64><<<grid, 256, 0, stream>>>(dy, dx, db, (int)M, N, seed, thr,
                                                           dropout_scale16(thr), graph_seed_ofs());
}

void transpose(const bf16_t* src, bf16_t* dst, int R, int C, int ldd, hipStream_t stream) {
  transpose_kernel<<<dim3(cdiv(C, 128), cdiv(ldd, 128)), 256, 0, stream>>>(src, dst, R, C, ldd);
}

void bias_grad(const bf16_t* dy, float* db, long M, int N, hipStream_t stream, long ld) {
  const int cvb = bias_cvb(N);
  const dim3 grid = bias_grid(M, N, cvb);
  if (ld <= 0) ld = N;
  if (cvb == 32)
    bias_grad_kernel<32><<<grid, 256, 0, stream>>>(dy, db, (int)M, N, ld);
  else
    bias_grad_kernel<64><<<grid, 256, 0, stream>>>(dy, db, (int)M, N, ld);
}

}  // namespace mg
