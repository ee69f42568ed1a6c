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
//  * v_mfma_f32_16x16x32_bf16, BK = 64, tile configs chosen per shape:
//      T128: 128x128 tile, 4 waves (2x2) of 64x64, 64 KiB LDS -> 2 workgroups / CU
//      T256: 256x256 tile, 8 waves (2x4) of 128x64, 128 KiB LDS -> 1 workgroup / CU (2 waves/SIMD)
//      T2x1: 256x128 tile, 8 waves (4x2) of 64x64, 96 KiB LDS
//  * LDS-DMA staging (buffer_load_dwordx4 ... lds): global -> LDS without VGPRs, tile k+1 in flight
//    while tile k is multiplied (2-stage ring, one vmcnt(0) + barrier per K-step).  The buffer range
//    check zero-fills every row / column / K tail, so no tail code runs in the main loop.
//  * k-contiguous tiles: 128-B rows, chunk ^ (row & 7) swizzle -> conflict-free ds_read_b128;
//    m/n-contiguous tiles: [64 k][128] half-images with 256-B rows and the T10(b) swizzle, read by
//    ds_read_b64_tr_b16 (hardware transpose) -> all three layouts without a transpose pass in HBM.
//    The swizzle is applied to the DMA *source* address (the LDS image of an LDS-DMA is lane-linear).
//  * operands swapped in the MFMA (C^T = B'^T A'^T): each lane holds 4 consecutive n of one row m,
//    so epilogue stores are 8 B (bf16) / 16 B (fp32).
//  * XCD-aware bijective block remap + GROUP_M ordering (blocks sharing A rows share an XCD's L2).
//  * epilogues: none | +bias | +bias,GELU (pre-activation also stored) |
//    resid + dropout(acc + bias) (Philox mask, same element mapping as elementwise.hip) |
//    acc * GELU'(pre) | fp32 accumulate (the main-grad buffer), split-K via LDS-staged atomics.
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 64;
constexpr int GROUP_M = 8;
constexpr uint32_t kOOB = 0xFFFFFFF0u;

template <int BM_, int BN_, int NWM_, int NWN_, int STAGES_ = 2>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, NWM = NWM_, NWN = NWN_, STAGES = STAGES_;
  static constexpr int NW = NWM * NWN, NT = NW * 64;
  static constexpr int WTM = BM / NWM, WTN = BN / NWN;  // wave tile
  static constexpr int FM = WTM / 16, FN = WTN / 16;    // 16x16 MFMA tiles per wave
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int SMEM = STAGES * STAGE;
  // LDS-DMA wave-instructions one wave issues per K-step (for the counted vmcnt)
  static constexpr int DMA_PER_STEP = BM / 8 / NW + BN / 8 / NW;
};
using T128 = Cfg<128, 128, 2, 2>;
using T256 = Cfg<256, 256, 2, 4>;
using T2x1 = Cfg<256, 128, 4, 2, 3>;  // 3-stage ring: two K-steps in flight, 144 KiB

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  long lda, ldb, ldc;
  int M, N, K;     // C is M x N (store bounds), reduction K
  int a_ext;       // load extent of A' along m (rows for k-contig, row length for m-contig)
  int b_ext;       // load extent of B' along n
  int ka, kb;      // A' (resp. B') reads as zero for k >= ka (kb)
  const bf16_t* bias;
  bf16_t* aux;     // GELU pre-activation: written (EPI 2) or read (EPI 4); [M, ldc]
  const bf16_t* resid;
  uint64_t seed;
  uint32_t thr;
  float scale;
  int tiles_m, tiles_n;
  int splits, kchunk;         // split-K (fp32-accumulate layout only): K range per split
  uint32_t a_bytes, b_bytes;  // buffer-resource extents (out-of-range reads return 0)
};

static int g_variant = 0;  // 0 auto, 1 force T128, 2 force T256, 3 force T2x1

MG_DEVICE int swz_mn(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// ---- LDS-DMA staging of one operand tile (R rows/cols of the m|n dimension x BK) by NW waves.
// Each buffer_load ... lds wave-instruction writes 1 KiB at (wave-uniform base + lane*16).
template <bool KC, int R, int NW>
MG_DEVICE void dma_tile(char* lds, __amdgpu_buffer_rsrc_t rs, long ld, int r0, int ext, int k0,
                        int kvalid, int wid, int lane) {
  constexpr int PER = R / 8 / NW;  // 1-KiB blocks per wave (R*128 B per tile)
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = wid * PER + i;
    uint32_t off;
    if constexpr (KC) {  // [R rows][128 B]: block = 8 rows x 8 chunks
      const int row = 8 * j + (lane >> 3), ch = (lane & 7) ^ (row & 7);
      const int gr = r0 + row, gk = k0 + ch * 8;
      off = (gr < ext && gk < kvalid) ? (uint32_t)(((long)gr * ld + gk) * 2) : kOOB;
    } else {  // R/128 half-images [64 k][256 B]: block = 4 k-rows x 16 chunks
      const int half = j >> 4, jj = j & 15;
      const int row = 4 * jj + (lane >> 4), ch = (lane & 15) ^ swz_mn(row);
      const int gk = k0 + row, gc = r0 + half * 128 + ch * 8;
      off = (gk < kvalid && gc < ext) ? (uint32_t)(((long)gk * ld + gc) * 2) : kOOB;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + j * 1024), 16, off, 0, 0, 0);
  }
}

// ---- fragment read for 16-wide subtile sb, k-step ks (32 k)
template <bool KC>
MG_DEVICE bf16x8 frag(const char* lds, int sb, int ks, int lane) {
  if constexpr (KC) {
    const int row = sb * 16 + (lane & 15);
    const int ch = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((ch ^ (row & 7)) << 4));
  } else {
    const char* img = lds + (sb >> 3) * 16384;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int chk = (sb & 7) * 2 + (p >> 1);
    const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
    const char* a0 = img + r0 * 256 + ((chk ^ swz_mn(r0)) << 4) + (p & 1) * 8;
    const char* a1 = img + r1 * 256 + ((chk ^ swz_mn(r1)) << 4) + (p & 1) * 8;
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <class CF, bool AK, bool BKC, int EPI, bool OUTF32>
__global__ __launch_bounds__(CF::NT, 2) void gemm_kernel(const GemmArgs args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / CF::NWN, wn = wid % CF::NWN;

  // XCD-aware bijective remap, then split index, then GROUP_M swizzle over output tiles
  const int nblk = args.tiles_m * args.tiles_n * args.splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wgs = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int ntiles = args.tiles_m * args.tiles_n;
  const int split = wgs / ntiles;  // split slowest: neighbours on an XCD share a K range (L2 reuse)
  const int wg = wgs % ntiles;
  const int group = GROUP_M * args.tiles_n;
  const int first_m = (wg / group) * GROUP_M;
  const int gm = min(args.tiles_m - first_m, GROUP_M);
  const int pid_m = first_m + (wg % group) % gm;
  const int pid_n = (wg % group) / gm;
  const int m0 = pid_m * CF::BM, n0 = pid_n * CF::BN;

  f32x4 acc[CF::FM][CF::FN];
#pragma unroll
  for (int i = 0; i < CF::FM; ++i)
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kbeg = split * args.kchunk;
  const int nk = (min(args.K, kbeg + args.kchunk) - kbeg + BK - 1) / BK;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)args.A, 0, args.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)args.B, 0, args.b_bytes, 0x00020000);
  // prologue: STAGES-1 tiles in flight
#pragma unroll
  for (int st = 0; st < CF::STAGES - 1; ++st) {
    if (st < nk) {
      char* dst = smem + st * CF::STAGE;
      dma_tile<AK, CF::BM, CF::NW>(dst, rsa, args.lda, m0, args.a_ext, kbeg + st * BK, args.ka, wid, lane);
      dma_tile<BKC, CF::BN, CF::NW>(dst + CF::A_BYTES, rsb, args.ldb, n0, args.b_ext, kbeg + st * BK, args.kb, wid, lane);
    }
  }
  if constexpr (CF::STAGES == 3) {
    if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CF::DMA_PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt % CF::STAGES) * CF::STAGE;
    const char* sb = sa + CF::A_BYTES;
    const int kn = kt + CF::STAGES - 1;  // tile to issue now
    if (kn < nk) {  // its stage was last read in iteration kt-1: free since that barrier
      char* dst = smem + (kn % CF::STAGES) * CF::STAGE;
      const int k1 = kbeg + kn * BK;
      dma_tile<AK, CF::BM, CF::NW>(dst, rsa, args.lda, m0, args.a_ext, k1, args.ka, wid, lane);
      dma_tile<BKC, CF::BN, CF::NW>(dst + CF::A_BYTES, rsb, args.ldb, n0, args.b_ext, k1, args.kb, wid, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[CF::FM], fb[CF::FN];
#pragma unroll
      for (int i = 0; i < CF::FM; ++i) fa[i] = frag<AK>(sa, wm * CF::FM + i, ks, lane);
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) fb[j] = frag<BKC>(sb, wn * CF::FN + j, ks, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    // tile kt+1 must have landed (this wave's DMA), every wave's LDS reads of stage kt retired;
    // with 3 stages the DMA of tile kt+2 stays in flight across the barrier (counted vmcnt).
    if constexpr (CF::STAGES == 3) {
      if (kn < nk) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(CF::DMA_PER_STEP) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }

  if constexpr (OUTF32) {
    if (args.splits > 1) {
      // split-K: fp32 atomics into C.  Each wave stages its tile through LDS 32 rows at a time
      // (row stride WTN+4 floats: conflict-free ds_write_b128), then every atomic
      // wave-instruction adds WTN contiguous floats of one row (256 B: the full-rate shape).
      constexpr int RS = CF::WTN + 4;
      float* ct = reinterpret_cast<float*>(smem) + wid * 32 * RS;
      float* C = reinterpret_cast<float*>(args.C);
#pragma unroll
      for (int pass = 0; pass < CF::FM / 2; ++pass) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < CF::FN; ++j)
            *reinterpret_cast<f32x4*>(ct + (ii * 16 + (lane & 15)) * RS + j * 16 + (lane >> 4) * 4) =
                acc[pass * 2 + ii][j];
        __syncthreads();
        for (int c = lane; c < CF::WTN; c += 64) {
          const int n = n0 + wn * CF::WTN + c;
          for (int r = 0; r < 32; ++r) {
            const int m = m0 + wm * CF::WTM + pass * 32 + r;
            if (m < args.M && n < args.N) atomicAdd(C + (long)m * args.ldc + n, ct[r * RS + c]);
          }
        }
        __syncthreads();
      }
      return;
    }
  }
  // ---- epilogue: lane holds C[m][n..n+3]
  const int nlim = (EPI == 0 && !OUTF32) ? (int)args.ldc : args.N;
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
    const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
    if (m >= args.M) continue;
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) {
      const int n = n0 + wn * CF::WTN + j * 16 + (lane >> 4) * 4;
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

template <class CF, bool AK, bool BKC, int EPI, bool OUTF32>
void launch(GemmArgs a, hipStream_t stream) {
  a.tiles_m = cdiv(a.M, CF::BM);
  a.tiles_n = cdiv(a.N, CF::BN);
  a.splits = 1;
  a.kchunk = cdiv(a.K, BK) * BK;
  if (OUTF32) {  // weight gradient: small outputs, huge K -> split K until the chip is full
    const int tiles = a.tiles_m * a.tiles_n;
    const int slots = 256 * (CF::SMEM <= 80 * 1024 ? 2 : 1);
    int sp = tiles >= (3 * slots) / 4 ? 1 : std::min(16, cdiv(slots, tiles));
    const int nkt = cdiv(a.K, BK);
    sp = std::min(sp, nkt);
    a.kchunk = cdiv(nkt, sp) * BK;
    a.splits = cdiv(a.K, a.kchunk);
  }
  const int grid = a.tiles_m * a.tiles_n * a.splits;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_kernel<CF, AK, BKC, EPI, OUTF32>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, CF::SMEM);
    attr_set = true;
  }
  gemm_kernel<CF, AK, BKC, EPI, OUTF32><<<grid, CF::NT, CF::SMEM, stream>>>(a);
}

// Tile config per shape (measured, bench/bench_gemm.py): the 256x256 tile (1 workgroup/CU, more
// MFMA work per LDS byte) wins once it has >= 2 full rounds of tiles on the 256 CUs (LM head:
// 1.57 vs 1.87 ms); otherwise 128x128 (2 workgroups/CU, finer quantisation) is as fast or faster,
// and always for the split-K weight gradient.
int pick_config(int M, int N, bool outf32) {
  if (g_variant) return g_variant;
  if (outf32) return 1;
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  return t256 >= 512 ? 2 : 1;
}

template <bool AK, bool BKC, int EPI, bool OUTF32>
void dispatch(const GemmArgs& a, hipStream_t stream) {
  switch (pick_config(a.M, a.N, OUTF32)) {
    case 2: launch<T256, AK, BKC, EPI, OUTF32>(a, stream); break;
    case 3: launch<T2x1, AK, BKC, EPI, OUTF32>(a, stream); break;
    default: launch<T128, AK, BKC, EPI, OUTF32>(a, stream); break;
  }
}

}  // namespace

namespace mg {

void gemm_set_variant(int v) { g_variant = v; }
int gemm_get_variant() { return g_variant; }

// layout: 0 = NT (fwd), 1 = NN (dgrad), 2 = TN (wgrad, fp32 accumulate into C)
void gemm(int layout, int epi, const bf16_t* A, const bf16_t* B, void* C, long lda, long ldb,
          long ldc, int M, int N, int K, int a_ext, int b_ext, int ka, int kb, const bf16_t* bias,
          bf16_t* aux, const bf16_t* resid, float p, uint64_t seed, hipStream_t stream,
          size_t a_bytes, size_t b_bytes) {
  GemmArgs a;
  a.a_bytes = (uint32_t)std::min<size_t>(a_bytes, 0xFFFFFF00u);
  a.b_bytes = (uint32_t)std::min<size_t>(b_bytes, 0xFFFFFF00u);
  a.A = A; a.B = B; a.C = C; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K; a.a_ext = a_ext; a.b_ext = b_ext; a.ka = ka; a.kb = kb;
  a.bias = bias; a.aux = aux; a.resid = resid; a.seed = seed;
  a.thr = p > 0.f ? dropout_threshold(p) : 0u;
  a.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  a.tiles_m = a.tiles_n = a.splits = 1;
  a.kchunk = K;
  if (layout == 0) {
    if (epi == 0) dispatch<true, true, 0, false>(a, stream);
    else if (epi == 1) dispatch<true, true, 1, false>(a, stream);
    else if (epi == 2) dispatch<true, true, 2, false>(a, stream);
    else dispatch<true, true, 3, false>(a, stream);
  } else if (layout == 1) {
    if (epi == 4) dispatch<true, false, 4, false>(a, stream);
    else dispatch<true, false, 0, false>(a, stream);
  } else {
    dispatch<false, false, 0, true>(a, stream);
  }
}

}  // namespace mg
