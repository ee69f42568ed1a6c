// bf16 MFMA GEMM with fused epilogues for gfx950 (CDNA4, MI355X).
//
// Replaces every nn.Linear / nn.MultiheadAttention projection of the reference
// (/root/reference/mingpt/model.py:138,147-154,180-181,249) in forward, data-gradient and
// weight-gradient form:
//
//   C[m, n] = sum_k A'[m, k] * B'[k, n]
//   layout NT: A' = A[M,K] (k contiguous), B' = B[N,K]^T (k contiguous)   -> forward  y = x W^T
//   layout NN: A' = A[M,K] (k contiguous), B' = B[K,N]  (n contiguous)    -> dgrad   dx = dy W
//   layout TN: A' = A[K,M]^T (m contiguous), B' = B[K,N] (n contiguous)  -> wgrad   dW += dy^T x
//
// Design (see /opt/skills/guides/cdna_hip_programming.md §5):
//  * v_mfma_f32_16x16x32_bf16; block tile 128x128x64, 4 waves (2x2), each wave a 64x64 C tile of
//    4x4 MFMA tiles (64 fp32 accumulators per lane).
//  * LDS double buffer (2 x 32 KiB); global->register->LDS staging with the loads for tile k+1
//    issued before the MFMAs of tile k and written after them (one barrier per K-step).
//  * k-contiguous tiles use 128-B rows with an XOR swizzle (chunk ^ row&7) so the ds_read_b128
//    fragment reads are bank-conflict-free; m/n-contiguous tiles use 256-B rows with the
//    T10 (b) swizzle and are read with ds_read_b64_tr_b16 (hardware transpose), so the same kernel
//    serves all three layouts without any transpose pass in HBM.
//  * operands are swapped in the MFMA (C^T = B'^T A'^T) so each lane ends up holding 4
//    consecutive n of one row m: 8-byte bf16 / 16-byte fp32 epilogue stores.
//  * XCD-aware bijective block remap + GROUP_M ordering: blocks that share A rows run on the same
//    XCD (private 4 MiB L2).
//  * epilogues: none | +bias | +bias,GELU (pre-activation also stored) |
//    resid + dropout(acc + bias) (Philox mask, same element mapping as elementwise.hip) |
//    acc * GELU'(pre) | fp32 accumulate (C += acc, the main-grad buffer).
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;     // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;  // A + B
constexpr int GROUP_M = 8;

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  long lda, ldb, ldc;
  int M, N, K;     // C is M x N (store bounds), reduction K
  int a_ext;       // load extent of A' along m (rows for k-contig, row length for m-contig)
  int b_ext;       // load extent of B' along n
  int ka, kb;      // zero-fill A' (resp. B') for k >= ka (kb)
  const bf16_t* bias;
  bf16_t* aux;     // GELU pre-activation: written (EPI_GELU) or read (EPI_GELU_BWD); [M, ldc]
  const bf16_t* resid;
  uint64_t seed;
  uint32_t thr;
  float scale;
  int tiles_m, tiles_n;
  int splits, kchunk;  // split-K (fp32-accumulate layout only): K range per split, multiple of BK
};

MG_DEVICE int swz_mn(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// ---- staging: global -> registers (4 x 16 B per thread per operand tile)
template <bool KC>
MG_DEVICE void load_tile(uint4 (&reg)[4], const bf16_t* __restrict__ base, long ld, int r0, int ext,
                         int k0, int kvalid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + 256 * i;
    if constexpr (KC) {  // 128 rows (m or n) x 8 chunks of 8 k
      const int row = idx >> 3, ch = idx & 7;
      const int gr = min(r0 + row, ext - 1);
      const int gk = k0 + ch * 8;
      reg[i] = gk < kvalid ? ld16(base + (long)gr * ld + gk) : make_uint4(0, 0, 0, 0);
    } else {  // 64 k-rows x 16 chunks of 8 (m or n)
      const int kr = idx >> 4, ch = idx & 15;
      const int gk = k0 + kr;
      const int gc = min(r0 + ch * 8, ext - 8);
      reg[i] = gk < kvalid ? ld16(base + (long)gk * ld + gc) : make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KC>
MG_DEVICE void store_tile(char* lds, const uint4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + 256 * i;
    if constexpr (KC) {
      const int row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4*>(lds + row * 128 + ((ch ^ (row & 7)) << 4)) = reg[i];
    } else {
      const int kr = idx >> 4, ch = idx & 15;
      *reinterpret_cast<uint4*>(lds + kr * 256 + ((ch ^ swz_mn(kr)) << 4)) = reg[i];
    }
  }
}

// ---- fragment reads for one 16-wide subtile sb and k-step ks (32 k)
template <bool KC>
MG_DEVICE bf16x8 frag(const char* lds, int sb, int ks, int lane) {
  if constexpr (KC) {
    const int row = sb * 16 + (lane & 15);
    const int ch = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((ch ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int chk = sb * 2 + (p >> 1);
    const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
    const char* a0 = lds + r0 * 256 + ((chk ^ swz_mn(r0)) << 4) + (p & 1) * 8;
    const char* a1 = lds + r1 * 256 + ((chk ^ swz_mn(r1)) << 4) + (p & 1) * 8;
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <bool AK, bool BKC, int EPI, bool OUTF32>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective remap, then GROUP_M swizzle
  const int nblk = args.tiles_m * args.tiles_n * args.splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wgs = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int split = wgs % args.splits;
  const int wg = wgs / args.splits;
  const int group = GROUP_M * args.tiles_n;
  const int first_m = (wg / group) * GROUP_M;
  const int gm = min(args.tiles_m - first_m, GROUP_M);
  const int pid_m = first_m + (wg % group) % gm;
  const int pid_n = (wg % group) / gm;
  const int m0 = pid_m * BM, n0 = pid_n * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kbeg = split * args.kchunk;
  const int nk = (min(args.K, kbeg + args.kchunk) - kbeg + BK - 1) / BK;
  uint4 ra[4], rb[4];
  load_tile<AK>(ra, args.A, args.lda, m0, args.a_ext, kbeg, args.ka);
  load_tile<BKC>(rb, args.B, args.ldb, n0, args.b_ext, kbeg, args.kb);
  store_tile<AK>(smem, ra);
  store_tile<BKC>(smem + TILE_BYTES, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * STAGE_BYTES;
    const char* sb = sa + TILE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<AK>(ra, args.A, args.lda, m0, args.a_ext, kbeg + (kt + 1) * BK, args.ka);
      load_tile<BKC>(rb, args.B, args.ldb, n0, args.b_ext, kbeg + (kt + 1) * BK, args.kb);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag<AK>(sa, wm * 4 + i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag<BKC>(sb, wn * 4 + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* dst = smem + ((kt + 1) & 1) * STAGE_BYTES;
      store_tile<AK>(dst, ra);
      store_tile<BKC>(dst + TILE_BYTES, rb);
    }
    __syncthreads();
  }

  if constexpr (OUTF32) {
    if (args.splits > 1) {
      // split-K: fp32 atomics into C.  Stage each wave's 64x64 tile through LDS (row stride 68
      // floats: conflict-free ds_write_b128) in two 32-row halves, then every atomic
      // wave-instruction adds 64 contiguous floats of one row (256 B: the full-rate shape).
      float* ct = reinterpret_cast<float*>(smem) + wid * 32 * 68;
      float* C = reinterpret_cast<float*>(args.C);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *reinterpret_cast<f32x4*>(ct + (ii * 16 + (lane & 15)) * 68 + j * 16 + (lane >> 4) * 4) =
                acc[half * 2 + ii][j];
        __syncthreads();
        const int n = n0 + wn * 64 + lane;
        for (int r = 0; r < 32; ++r) {
          const int m = m0 + wm * 64 + half * 32 + r;
          if (m < args.M && n < args.N) atomicAdd(C + (long)m * args.ldc + n, ct[r * 68 + lane]);
        }
        __syncthreads();
      }
      return;
    }
  }
  // ---- epilogue: lane holds C[m][n..n+3]
  const int nlim = (EPI == 0 && !OUTF32) ? (int)args.ldc : args.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= args.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
      if (n >= nlim) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const long off = (long)m * args.ldc + n;
      if constexpr (OUTF32) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(args.C) + off);
        float4 c = *cp;
        c.x += v[0]; c.y += v[1]; c.z += v[2]; c.w += v[3];
        *cp = c;
      } else {
        if constexpr (EPI == 1 || EPI == 2 || EPI == 3) {
          if (args.bias) {
            const uint2 bb = *reinterpret_cast<const uint2*>(args.bias + n);
            v[0] += bf2f(bb.x & 0xffffu); v[1] += bf2f(bb.x >> 16);
            v[2] += bf2f(bb.y & 0xffffu); v[3] += bf2f(bb.y >> 16);
          }
        }
        if constexpr (EPI == 2) {
          *reinterpret_cast<uint2*>(args.aux + off) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
        }
        if constexpr (EPI == 3) {
          if (args.thr) {
            const uint4 rnd = rand4(args.seed, ((uint64_t)m * args.N + n) >> 2);
            const uint32_t rr[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rr[r] >= args.thr ? v[r] * args.scale : 0.f;
          }
          const uint2 res = *reinterpret_cast<const uint2*>(args.resid + off);
          v[0] += bf2f(res.x & 0xffffu); v[1] += bf2f(res.x >> 16);
          v[2] += bf2f(res.y & 0xffffu); v[3] += bf2f(res.y >> 16);
        }
        if constexpr (EPI == 4) {
          const uint2 pa = *reinterpret_cast<const uint2*>(args.aux + off);
          v[0] *= gelu_grad(bf2f(pa.x & 0xffffu)); v[1] *= gelu_grad(bf2f(pa.x >> 16));
          v[2] *= gelu_grad(bf2f(pa.y & 0xffffu)); v[3] *= gelu_grad(bf2f(pa.y >> 16));
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(args.C) + off) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
}

template <bool AK, bool BKC, int EPI, bool OUTF32>
void launch(const GemmArgs& a, hipStream_t stream) {
  const int grid = a.tiles_m * a.tiles_n * a.splits;
  gemm_kernel<AK, BKC, EPI, OUTF32><<<grid, 256, 2 * STAGE_BYTES, stream>>>(a);
}

}  // namespace

namespace mg {

// layout: 0 = NT (fwd), 1 = NN (dgrad), 2 = TN (wgrad, fp32 accumulate into C)
void gemm(int layout, int epi, const bf16_t* A, const bf16_t* B, void* C, long lda, long ldb,
          long ldc, int M, int N, int K, int a_ext, int b_ext, int ka, int kb, const bf16_t* bias,
          bf16_t* aux, const bf16_t* resid, float p, uint64_t seed, hipStream_t stream) {
  GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K; a.a_ext = a_ext; a.b_ext = b_ext; a.ka = ka; a.kb = kb;
  a.bias = bias; a.aux = aux; a.resid = resid; a.seed = seed;
  a.thr = p > 0.f ? dropout_threshold(p) : 0u;
  a.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  a.tiles_m = cdiv(M, BM);
  a.tiles_n = cdiv(N, BN);
  a.splits = 1;
  a.kchunk = cdiv(K, BK) * BK;
  if (layout == 2) {  // weight gradient: small outputs, huge K -> split K until ~2 blocks per CU
    const int tiles = a.tiles_m * a.tiles_n;
    int sp = tiles >= 384 ? 1 : std::min(16, cdiv(512, tiles));
    const int nkt = cdiv(K, BK);
    sp = std::min(sp, nkt);
    a.kchunk = cdiv(nkt, sp) * BK;
    a.splits = cdiv(K, a.kchunk);
  }
  if (layout == 0) {
    if (epi == 0) launch<true, true, 0, false>(a, stream);
    else if (epi == 1) launch<true, true, 1, false>(a, stream);
    else if (epi == 2) launch<true, true, 2, false>(a, stream);
    else launch<true, true, 3, false>(a, stream);
  } else if (layout == 1) {
    if (epi == 4) launch<true, false, 4, false>(a, stream);
    else launch<true, false, 0, false>(a, stream);
  } else {
    launch<false, false, 0, true>(a, stream);
  }
}

}  // namespace mg
