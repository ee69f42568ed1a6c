// LayerNorm forward / backward for gfx950.
//
// Replaces the reference's three ATen LayerNorms per block (ln_1, ln_2, ln_ff:
// /root/reference/mingpt/model.py:176,178,248).  Layout: x is [M, D] bf16 row-major.
//
// Forward: two rows per wave, 8 rows per 256-thread block; each lane holds NV chunks of 8
// contiguous bf16 (16-B loads) of both rows, so a row is read from HBM exactly once and the
// two-pass (mean, then centred variance) statistics come from registers.  mean/rstd in fp32.
//
// Backward: same row mapping.  dx is produced per row (optionally + the residual-branch gradient);
// dgamma/dbeta are accumulated per wave in registers over a grid-stride loop, folded across the
// block's waves through LDS and added into the fp32 main-grad buffers with one atomic per column
// per block.
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w,
                                                     const bf16_t* __restrict__ b,
                                                     bf16_t* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int M, int D,
                                                     float eps) {
  // two rows per wave (rows r and r + 4 of the block's 8): both rows' loads are issued before
  // either is reduced, so a wave keeps twice the bytes in flight
  const int lane = threadIdx.x & 63;
  const long r0 = (long)blockIdx.x * 8 + (threadIdx.x >> 6);
  if (r0 >= M) return;
  const long rows[2] = {r0, r0 + 4 < M ? r0 + 4 : r0};
  const bool two = r0 + 4 < M;
  uint4 raw[2][NV];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      raw[u][i] = c < D ? ld16(x + rows[u] * D + c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) break;
    const long row = rows[u];
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      unpack8(raw[u][i], v[i]);  // zero past D
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
    const float mu = wave_sum(s) / D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[i][j] - mu;
          ss += d * d;
        }
      }
    }
    const float rs = rsqrtf(wave_sum(ss) / D + eps);
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
    bf16_t* yr = y + row * D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
        float wf[8], bf[8], o[8];
        unpack8(ld16(w + c), wf);
        unpack8(ld16(b + c), bf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mu) * rs * wf[j] + bf[j];
        st16(yr + c, pack8(o));
      }
    }
  }
}

// DROP: the residual-dropout backward of the branch that produced this LN's input is fused in
// (the consumer of dx in the step: /root/reference/mingpt/model.py:187-188's residual adds).  Besides
// dx, the kernel writes dz = dropout'(bf16(dx)) (the same 16-bit mask as the forward's GEMM
// epilogue, common.h rowdrop8) and accumulates dz's fp32 column sums -- the branch's bias gradient
// -- into a third partial row; the separate dropout_bias_grad pass (one more 2-byte read per
// element) is gone.
struct LnDrop {
  bf16_t* dz;
  uint64_t seed;
  const uint64_t* sofs;
  uint32_t thr;
  float scale;
};

template <int NV, bool DROP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy,
                                                     const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const bf16_t* __restrict__ dres,
                                                     bf16_t* __restrict__ dx,
                                                     float* __restrict__ part, int M, int D, const LnDrop dr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int NP = DROP ? 3 : 2;  // partial row: [dgamma | dbeta (| dbias)]
  float zacc[DROP ? NV : 1][8];
#pragma unroll
  for (int i = 0; i < (DROP ? NV : 1); ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) zacc[i][j] = 0.f;
  const uint64_t dseed = DROP ? eff_seed(dr.seed, dr.sofs) : 0;
  // rows are held PACKED (bf16 x 8 per uint4) between load and use: two rows of x, dy and the
  // residual gradient in flight cost 3 x 2 x NV x 4 registers instead of twice that as floats
  // (NV = 4, gpt2-xl's D = 1600, had 504 registers -> one wave per SIMD)
  float gacc[NV][8], bacc[NV][8];
  uint4 wraw[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    wraw[i] = c < D ? ld16(w + c) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gacc[i][j] = 0.f;
      bacc[i][j] = 0.f;
    }
  }
  // two rows per iteration: both rows' loads are issued before either is reduced, so each wave
  // keeps ~6 KB in flight instead of one row's dependent load -> reduce -> store chain
  const long stride = (long)gridDim.x * 8;
  for (long r0 = (long)blockIdx.x * 8 + wid; r0 < M; r0 += stride) {
    const long rows[2] = {r0, r0 + 4};
    uint4 xr[2][NV], gr[2][NV], rr[2][NV];
    float mu[2], rs[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long row = rows[u] < M ? rows[u] : rows[0];
      mu[u] = mean[row];
      rs[u] = rstd[row];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < D) {
          xr[u][i] = ld16(x + row * D + c);
          gr[u][i] = ld16(dy + row * D + c);
          if (dres) rr[u][i] = ld16(dres + row * D + c);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (rows[u] >= M) break;
      const long row = rows[u];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < D) {
          float xv[8], g[8], wf[8];
          unpack8(xr[u][i], xv);
          unpack8(gr[u][i], g);
          unpack8(wraw[i], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xh = (xv[j] - mu[u]) * rs[u];
            const float gw = g[j] * wf[j];
            s1 += gw;
            s2 += gw * xh;
            gacc[i][j] += g[j] * xh;
            bacc[i][j] += g[j];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        reg_fence(xr[u][i]);
        reg_fence(gr[u][i]);
        reg_fence(wraw[i]);
      }
      s1 = wave_sum(s1) / D;
      s2 = wave_sum(s2) / D;
      bf16_t* dxr = dx + row * D;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < D) {
          float xv[8], g[8], wf[8], o[8];
          unpack8(xr[u][i], xv);
          unpack8(gr[u][i], g);
          unpack8(wraw[i], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            o[j] = rs[u] * (g[j] * wf[j] - s1 - (xv[j] - mu[u]) * rs[u] * s2);
          if (dres) {  // fused residual-branch gradient: dx = LN'(dy) + dres
            float rv[8];
            unpack8(rr[u][i], rv);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += rv[j];
          }
          const uint4 packed = pack8(o);
          st16(dxr + c, packed);
          if constexpr (DROP) {  // dz = dropout'(stored dx), its column sums (fp32)
            float z[8];
            unpack8(packed, z);
            rowdrop8(z, dseed, row, c, D, dr.thr, dr.scale);
            st16(dr.dz + row * D + c, pack8(z));
#pragma unroll
            for (int j = 0; j < 8; ++j) zacc[i][j] += z[j];
          }
        }
      }
    }
  }
  // fold the 4 waves' column partials through LDS, one plane at a time, and store the block's
  // partial row [dgamma | dbeta (| dbias)] with plain stores; ln_colsum_kernel adds the blocks up
  // (a single-stage atomic fold put every block's atomics on the same 2D addresses).  One plane
  // of LDS (16 D bytes, 64 KiB at D = 4096) for any NP: all planes at once needed 48 D bytes with
  // the dropout plane, past the 160 KiB LDS for D > 3413.
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][D]
  float* prow = part + (long)blockIdx.x * NP * D;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    if (k) __syncthreads();  // the previous plane's readers are done
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wid * D + c + j] = k == 0 ? gacc[i][j] : k == 1 ? bacc[i][j] : zacc[DROP ? i : 0][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) prow[k * D + c] = red[c] + red[D + c] + red[2 * D + c] + red[3 * D + c];
  }
}

// dw += sum over blocks of part[:, :D], db += ... part[:, D:].  Block = 64 columns x 4 waves over a
// 32-row chunk of the G partial rows (8 independent loads per lane: latency, not bandwidth, is
// what this pass pays); one atomic per column per block (G / 32 per address).
__global__ __launch_bounds__(256) void ln_colsum_kernel(const float* __restrict__ part, int G, int D, int NP,
                                                        float* __restrict__ dw, float* __restrict__ db,
                                                        float* __restrict__ dzb) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * 32;
  float s = 0.f;
  if (c < NP * D) {
    const int r1 = min(G, r0 + 32);
    for (int r = r0 + wid; r < r1; r += 4) s += part[(long)r * NP * D + c];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && c < NP * D) {
    const float v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (c < D) atomicAdd(dw + c, v);
    else if (c < 2 * D) atomicAdd(db + c - D, v);
    else atomicAdd(dzb + c - 2 * D, v);
  }
}

}  // namespace

namespace mg {

// >= 32 rows per block (4 waves x 2 rows x >= 4 iterations) up to 1024 blocks
// One resident wave of blocks: the kernel grid-strides over rows, and a grid of more blocks than
// fit the CUs at once (1024 at D = 768, where 150 VGPRs leave room for 3 blocks per CU = 768)
// ran a second, one-third-full round.  Occupancy from the runtime for the instantiation (D, and
// with or without the fused dropout plane) the launch selects.
template <int NV, bool DROP>
static int ln_bwd_resident() {
  static int n = 0;
  if (!n) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)ln_bwd_kernel<NV, DROP>, 256,
                                                       sizeof(float) * 4 * NV * 512);
    n = std::max(1, cus * std::max(1, per_cu));
  }
  return n;
}

template <bool DROP>
static int ln_bwd_cap(int D) {
  return D <= 512 ? ln_bwd_resident<1, DROP>() : D <= 1024 ? ln_bwd_resident<2, DROP>()
         : D <= 2048 ? ln_bwd_resident<4, DROP>() : ln_bwd_resident<8, DROP>();
}

int ln_bwd_grid(int M, int D, bool drop) {
  const int cap = drop ? ln_bwd_cap<true>(D) : ln_bwd_cap<false>(D);
  return std::max(1, std::min(M / 32, cap));
}

#define MG_LN_DISPATCH(KERNEL, ...)                                                   \
  do {                                                                                \
    if (D <= 512) KERNEL<1><<<grid, 256, smem, stream>>>(__VA_ARGS__);                \
    else if (D <= 1024) KERNEL<2><<<grid, 256, smem, stream>>>(__VA_ARGS__);          \
    else if (D <= 2048) KERNEL<4><<<grid, 256, smem, stream>>>(__VA_ARGS__);          \
    else KERNEL<8><<<grid, 256, smem, stream>>>(__VA_ARGS__);                         \
  } while (0)

void layernorm_fwd(const bf16_t* x, const bf16_t* w, const bf16_t* b, bf16_t* y, float* mean,
                   float* rstd, int M, int D, float eps, hipStream_t stream) {
  const int grid = cdiv(M, 8);  // 8 rows per block: two per wave
  const size_t smem = 0;
  MG_LN_DISPATCH(ln_fwd_kernel, x, w, b, y, mean, rstd, M, D, eps);
}

void layernorm_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* w, const float* mean,
                   const float* rstd, const bf16_t* dres, bf16_t* dx, float* dw, float* db,
                   float* workspace, int M, int D, hipStream_t stream, bf16_t* dz, float* dzb, float p,
                   uint64_t seed) {
  const bool drop = dz != nullptr;
  const int grid = ln_bwd_grid(M, D, drop);
  const int NP = drop ? 3 : 2;
  const size_t smem = sizeof(float) * 4 * D;  // one partial plane at a time
  const uint32_t thr = drop ? dropout_threshold16(p) : 0u;
  const LnDrop dr{dz, seed, graph_seed_ofs(), thr, dropout_scale16(thr)};
#define MG_LN_BWD(NV)                                                                                   \
  if (drop) ln_bwd_kernel<NV, true><<<grid, 256, smem, stream>>>(dy, x, w, mean, rstd, dres, dx, workspace, M, D, dr); \
  else ln_bwd_kernel<NV, false><<<grid, 256, smem, stream>>>(dy, x, w, mean, rstd, dres, dx, workspace, M, D, dr);
  if (D <= 512) { MG_LN_BWD(1) }
  else if (D <= 1024) { MG_LN_BWD(2) }
  else if (D <= 2048) { MG_LN_BWD(4) }
  else { MG_LN_BWD(8) }
#undef MG_LN_BWD
  ln_colsum_kernel<<<dim3(cdiv(NP * D, 64), cdiv(grid, 32)), 256, 0, stream>>>(workspace, grid, D, NP, dw, db, dzb);
}

// floats of partial [dgamma | dbeta (| dbias)] rows layernorm_bwd needs
size_t layernorm_bwd_workspace(int M, int D, bool drop) {
  return (size_t)ln_bwd_grid(M, D, drop) * (drop ? 3 : 2) * D;
}

}  // namespace mg
