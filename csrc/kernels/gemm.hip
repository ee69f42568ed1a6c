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
//  * v_mfma_f32_16x16x32_bf16, BK = 64, tile configs chosen per shape (pick_config):
//      W4:   256x256 (or 256x192) tile, 4 waves (2x2) of 128x128 (128x96), 160 KiB LDS, one wave
//            per SIMD holding the whole register file (the default for every large shape)
//      T128: 128x128 tile, 4 waves (2x2) of 64x64, 64 KiB LDS -> 2 workgroups / CU (small outputs,
//            and weight gradients whose tile count quantises badly onto 256 CUs at 256^2)
//    (the 8-wave 256x256 ping-pong, 256x256 / 8-wave and 256x128 block configs of rounds 1-2 never
//    won a shape once W4 existed and were deleted in round 5; PERF.md)
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
//  * epilogues: none | +bias | +bias,GELU (GELU'(z) also stored: row-major, or in the W4 tiles'
//    fragment order straight from the registers, EPI 6) | resid + dropout(acc + bias) (counter-hash
//    row-block mask, common.h; the residual added in the fragment layout) | acc * GELU' (+ the fc
//    bias gradient's column sums; row-major EPI 4 or fragment-ordered EPI 7) | fp32 accumulate
//    (the main-grad buffer), split-K via atomics.  bf16 outputs leave through a per-wave LDS
//    staging as 16-byte pieces of whole rows (epilogue_staged).
#include "common.h"
#include "kernels.h"
#include <type_traits>


using namespace mg;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 64;
#ifndef MG_GROUP_M
#define MG_GROUP_M 8
#endif
constexpr int GROUP_M = MG_GROUP_M;  // row tiles per L2 group (blocks of a group share B column tiles)
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
};
using T128 = Cfg<128, 128, 2, 2>;

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
  const uint64_t* sofs;  // hipGraph mode: per-replay seed counter (common.h eff_seed), else nullptr
  uint32_t thr;
  float scale;
  int tiles_m, tiles_n;
  int splits, kchunk;         // split-K (fp32-accumulate layout only): K range per split
  uint64_t a_bytes, b_bytes;  // operand sizes; each block's descriptor spans <= 4 GiB from its origin
  unsigned long long* dbg;    // MG_GEMM_STAMPS diagnostic builds only: per-wave phase timestamps
  float* dbias;               // EPI 4: += column sums of the output (the bias gradient), or null
  int nt_out;                 // non-temporal bf16 output stores (see gemm() below)
};

static unsigned long long* g_dbg = nullptr;  // MG_GEMM_STAMPS builds: stamp buffer
static int g_variant = 0;  // 0 auto, 1 force T128, 5 force W4, 6 force W4 BN=192 (2-4: deleted configs)

// Chunk swizzle of the m/n-contiguous [64 k][256 B] half-images: rows 8 g + q (q < 4) of one
// transposed read get 8 distinct chunk pairs (conflict-free ds_read_b64_tr_b16), and bit 2 of the
// row is not used, so row r + 4 -- the second read of a fragment -- is the first one's address +
// 1024 (an immediate offset: no address VALU, which overflowed the MFMA gaps of the weight-gradient
// main loop: 1.54k vs 1.02k cycles per phase, tools/gemm_stamps.hip layout 2)
MG_DEVICE int swz_mn(int r) { return ((r & 3) << 2) | (((r >> 3) & 1) << 1); }

// ---- Buffer descriptor of K-tile t: base advanced to the tile's first k, extent shrunk with it,
// so per-lane offsets stay fixed while out-of-range rows (kOOB) and the buffer end still read 0.
// The inputs are readfirstlane'd: provably uniform, hence no waterfall loop per buffer op.
MG_DEVICE __amdgpu_buffer_rsrc_t tile_rsrc(const char* base, uint32_t bytes, uint32_t step, int t) {
  const uint32_t adv = (uint32_t)t * step;
  const uint64_t p = reinterpret_cast<uint64_t>(base) + adv;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(adv < bytes ? bytes - adv : 0u);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// ---- LDS-DMA stager of one operand tile (R rows/cols of the m|n dimension x BK) by NW waves.
// Each buffer_load ... lds wave-instruction writes 1 KiB at (wave-uniform base + lane*16).
// Per-lane source offsets are computed once; a K-tile costs one descriptor (SALU) plus, per piece,
// an M0 write and the load.  Per-lane k checks run only on K-tiles that cross the valid k extent.
// HS: byte stride between the two 128-column half-images of an m/n-contiguous operand (16 KiB:
// contiguous halves; W4's slot-unrolled loop interleaves the ring's slots inside each half)
template <bool KC, int R, int NW, int HS = 16384>
struct Stager {
  static constexpr int PER = R / 8 / NW;  // 1-KiB pieces per wave (R*128 B per tile)
  uint32_t voff[PER];
  const char* ptr;  // operand base
  const char* base;
  uint64_t total;  // operand bytes (may exceed 4 GiB: the descriptor starts at the tile / split origin)
  uint32_t bytes, step;
  long ld;
  int kbeg, klim, tail_t, swid;

  // k-contiguous operands: per-lane offsets are relative to the tile's first row (the row origin is
  // in the descriptor base, see retarget), so they are the same for every tile; rows past the
  // operand read as zero through the descriptor extent (the operand buffer ends at its last row).
  // m/n-contiguous operands: absolute offsets with a per-lane column check.
  MG_DEVICE void init(const bf16_t* p, uint64_t tot, long ld_, int r0, int ext, int kbeg_, int kvalid,
                      int kend, int wid, int lane) {
    ptr = reinterpret_cast<const char*>(p);
    total = tot;
    ld = ld_;
    kbeg = kbeg_;
    step = KC ? BK * 2 : (uint32_t)(BK * ld * 2);
    klim = min(kvalid, kend) - kbeg;
    tail_t = klim / BK;
    swid = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = wid * PER + i;
      if constexpr (KC) {  // [R rows][128 B]: block = 8 rows x 8 chunks
        const int row = 8 * j + (lane >> 3), ch = (lane & 7) ^ (row & 7);
        voff[i] = (uint32_t)(((long)row * ld + ch * 8) * 2);
      } else {  // R/128 half-images [64 k][256 B]: block = 4 k-rows x 16 chunks
        const int half = j >> 4, jj = j & 15;
        const int row = 4 * jj + (lane >> 4), ch = (lane & 15) ^ swz_mn(row);
        const int gc = r0 + half * 128 + ch * 8;
        voff[i] = gc < ext ? (uint32_t)(((long)row * ld + gc) * 2) : kOOB;
      }
    }
    retarget(r0);
  }
  // new tile origin (k-contiguous operands: scalar work only)
  MG_DEVICE void retarget(int r0) {
    const uint64_t o = KC ? (uint64_t)((long)r0 * ld + kbeg) * 2 : (uint64_t)kbeg * ld * 2;
    base = ptr + o;
    const uint64_t rest = total > o ? total - o : 0u;  // a block never reaches 4 GiB past its origin
    bytes = rest < 0xFFFFFF00u ? (uint32_t)rest : 0xFFFFFF00u;
  }
  // piece-level form for hand-interleaved schedules: descriptor once per tile, then piece(i)
  MG_DEVICE __amdgpu_buffer_rsrc_t rsrc(int t) const { return tile_rsrc(base, bytes, step, t); }
  // check = false: no per-lane k check, full K-tiles only (W4 visits its one partial K-tile first,
  // in the prologue)
  MG_DEVICE void piece(char* lds, __amdgpu_buffer_rsrc_t rs, int t, int i, bool check = true) const {
    const int j = swid * PER + i;
    uint32_t off = voff[i];
    if (check && t >= tail_t) {
      const int lane = threadIdx.x & 63;
      const int kpos = KC ? ((lane & 7) ^ ((lane >> 3) & 7)) * 8 : 4 * (j & 15) + (lane >> 4);
      off = kpos < klim - t * BK ? off : kOOB;
    }
    char* dst = KC ? lds + j * 1024 : lds + (j >> 4) * HS + (j & 15) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, off, 0, 0, 0);
  }
  MG_DEVICE void stage(char* lds, int t) const {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(base, bytes, step, t);
#pragma unroll
    for (int i = 0; i < PER; ++i) piece(lds, rs, t, i);
  }
};

// ---- transposing LDS read as inline asm.  Through the builtin, hipcc's wait-count pass sees an LDS
// read it cannot disambiguate from the in-flight LDS-DMA writes and puts s_waitcnt vmcnt(0) in
// front of it, which drains the DMA pipeline on every K-step of an m/n-contiguous operand (a third
// of the throughput).  The asm form is invisible to that pass, so every consumer makes the results
// valid itself: lds_ready() = s_waitcnt lgkmcnt(0) + a register tie, so no use (or copy) of a
// fragment is scheduled above the wait (scripts/mfma_hazards.py --lds checks the compiled code).
MG_DEVICE uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// ds_read_b64_tr_b16 with a constant byte offset in the instruction's offset field (no address VALU)
template <int OFF>
MG_DEVICE s16x4 ds_read_tr16_off(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int N>
MG_DEVICE void lds_ready(bf16x8 (&f)[N], bool wait = true) {
  if (wait) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

// ---- fragment read of a k-contiguous image for 16-wide subtile sb, k-step ks (32 k)
MG_DEVICE bf16x8 frag_kc(const char* lds, int sb, int ks, int lane) {
  const int row = sb * 16 + (lane & 15);
  const int ch = ks * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((ch ^ (row & 7)) << 4));
}

// frag with the k-step a template constant (W4): for m/n-contiguous images the k-step and the
// fragment's second row group go into the transposed reads' offset fields, so a fragment costs one
// address add (the ring slot base) and two reads
// HS: half-image stride; OFF: a constant byte offset (W4's slot-unrolled loop: the ring slot) that
// also goes into the offset field
template <bool KC, int KS, int HS = 16384, int OFF = 0>
MG_DEVICE bf16x8 frag_k(const char* lds, int sb, int lane) {
  if constexpr (KC) {
    return frag_kc(lds + OFF, sb, KS, lane);
  } else {
    const char* img = lds + (sb >> 3) * HS;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int chk = (sb & 7) * 2 + (p >> 1);
    const int r0 = 8 * g + q;  // + 32 KS (swz_mn ignores bits 2 and 5 of the row)
    const uint32_t a = lds_addr(img + r0 * 256 + ((chk ^ swz_mn(r0)) << 4) + (p & 1) * 8);
    const s16x4 x = ds_read_tr16_off<OFF + KS * 32 * 256>(a);
    const s16x4 y = ds_read_tr16_off<OFF + KS * 32 * 256 + 4 * 256>(a);
    const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// ---- LDS-staged bf16 epilogue.  The fragment layout gives each lane 4 columns of one row, so a
// direct store is an 8-byte global_store per lane and the store tail of a 256x256 tile is
// issue-bound (~2x the time of the same bytes in 16-byte stores, guide T21).  Each wave instead
// writes its finished fragments into its own LDS region (no workgroup barrier: the region is
// private and a wave's LDS ops complete in order), reads them back as 8 consecutive columns per
// lane and stores / loads side inputs with 16-byte accesses along whole wave-tile rows.
// Work that needs the fragment layout (bias, GELU, the row-block dropout mask) runs before the
// staging; the residual add / GELU' multiply read their side input after it, on fp32 staged values,
// so the rounding is identical to the direct form.
constexpr int stage_chf(int fm, int frag_row_bytes, int budget) {
  int c = fm;
  while (c > 1 && c * frag_row_bytes > budget) c >>= 1;
  return c;
}

MG_DEVICE uint4 load8(const bf16_t* p, int valid) {  // 8 bf16 at p, elements >= valid read as 0
  if (valid >= 8) return *reinterpret_cast<const uint4*>(p);
  uint16_t t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = e < valid ? p[e] : (uint16_t)0;
  return make_uint4(t[0] | (uint32_t)t[1] << 16, t[2] | (uint32_t)t[3] << 16, t[4] | (uint32_t)t[5] << 16,
                    t[6] | (uint32_t)t[7] << 16);
}

MG_DEVICE void store8(bf16_t* p, uint4 v, int valid) {
  if (valid >= 8) {
    *reinterpret_cast<uint4*>(p) = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (e < valid) p[e] = (uint16_t)(w[e >> 1] >> (16 * (e & 1)));
}

// EPI 4 bias gradient in the staged epilogue: a lane's 8-column piece index e % PR is the same in
// every pass when PR divides 64, so each lane keeps 8 running column sums of the fp32 outputs (before
// their bf16 rounding: one add per element; unpacking the rounded values cost the epilogue ~2.5 us
// per 256x256 tile at one wave per SIMD)
template <class CF>
constexpr bool staged_dbias() { return 64 % (CF::WTN / 8) == 0; }

// LDS -> global half of the staged epilogue for rows [mr, mr + 16 CHF) of the wave tile
// Whole-tile bf16 copy-out (no side input, no bounds checks): a lane's pieces are RPI rows apart
// at a fixed column, so its LDS and global addresses advance by constant strides (one base each,
// immediates / one add per piece), and the LDS reads go out G at a time ahead of their stores.
// Read-then-store per piece waited out each ds_read's latency before its store: 4.1-5.0k of the
// W4 tile's ~8k epilogue cycles at K = 768 (tools/gemm_stamps.hip with -DMG_GEMM_EPI_STAMPS).
template <int EPI, int S, int CHF, int PR, int IT, bool NT>
MG_DEVICE void staged_copy_out(const GemmArgs& args, const char* st, int mr, int nw, int lane) {
  constexpr int RPI = 64 / PR, G = 8;
  static_assert(IT % G == 0, "pieces per lane must be a multiple of the read group");
  const int r0 = lane / PR, p = lane % PR;
  const char* lrow = st + r0 * S + p * 16;
  const long off0 = (long)(mr + r0) * args.ldc + nw + p * 8;
  bf16_t* gc = reinterpret_cast<bf16_t*>(args.C) + off0;
  bf16_t* ga = EPI == 2 ? args.aux + off0 : nullptr;
  const long rs = (long)RPI * args.ldc;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int g0 = 0; g0 < IT; g0 += G) {
    uint4 y[G], z[EPI == 2 ? G : 1];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      y[u] = *reinterpret_cast<const uint4*>(lrow + (g0 + u) * RPI * S);
      if constexpr (EPI == 2) z[u] = *reinterpret_cast<const uint4*>(lrow + CHF * 16 * S + (g0 + u) * RPI * S);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long o = (long)(g0 + u) * rs;
      if constexpr (NT) {
        __builtin_nontemporal_store(v4u{y[u].x, y[u].y, y[u].z, y[u].w}, reinterpret_cast<v4u*>(gc + o));
        if constexpr (EPI == 2)
          __builtin_nontemporal_store(v4u{z[u].x, z[u].y, z[u].z, z[u].w}, reinterpret_cast<v4u*>(ga + o));
      } else {
        *reinterpret_cast<uint4*>(gc + o) = y[u];
        if constexpr (EPI == 2) *reinterpret_cast<uint4*>(ga + o) = z[u];
      }
    }
  }
}

// Whole-tile fp32-staged output with a bf16 side input (EPI 3: + residual, EPI 4: x GELU'), same
// addressing as staged_copy_out; the fp32 pieces are read G at a time ahead of their math and
// stores.  The side input `sd` was loaded for the whole pass before the staging.
template <class CF, int EPI, int S, int PR, int IT, bool NT>
MG_DEVICE void staged_side_out(const GemmArgs& args, const char* st, const uint4 (&sd)[IT], int mr, int nw,
                               int lane, float (&cs)[8]) {
  constexpr int RPI = 64 / PR, G = 2;  // 4 spilled at EPI 4 (the pass's side input holds 64 VGPRs)
  const int r0 = lane / PR, p = lane % PR;
  const char* lrow = st + r0 * S + p * 32;
  bf16_t* gc = reinterpret_cast<bf16_t*>(args.C) + (long)(mr + r0) * args.ldc + nw + p * 8;
  const long rs = (long)RPI * args.ldc;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int g0 = 0; g0 < IT; g0 += G) {
    float4 a[G], b[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      a[u] = *reinterpret_cast<const float4*>(lrow + (g0 + u) * RPI * S);
      b[u] = *reinterpret_cast<const float4*>(lrow + (g0 + u) * RPI * S + 16);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      float v[8] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w};
      if constexpr (EPI != 7) {  // EPI 7: GELU' was applied in the fragment layout, before the staging
        const uint4 sv = sd[g0 + u];
        const uint32_t w[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float s = bf2f((w[k >> 1] >> (16 * (k & 1))) & 0xffffu);
          v[k] = EPI == 3 ? v[k] + s : v[k] * s;
        }
      }
      if constexpr ((EPI == 4 || EPI == 7) && staged_dbias<CF>()) {
#pragma unroll
        for (int k = 0; k < 8; ++k) cs[k] += v[k];
      }
      const uint4 y = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
      bf16_t* dst = gc + (long)(g0 + u) * rs;
      if constexpr (NT) __builtin_nontemporal_store(v4u{y.x, y.y, y.z, y.w}, reinterpret_cast<v4u*>(dst));
      else *reinterpret_cast<uint4*>(dst) = y;
    }
  }
}

template <class CF, int EPI, bool F32, int S, int CHF, int PR, int IT, bool CHECK>
MG_DEVICE void staged_rows(const GemmArgs& args, const char* st, const uint4 (&sd)[F32 ? IT : 1], int mr,
                           int nw, int nlim, int lane, float (&cs)[8]) {
  if constexpr (!F32 && !CHECK && 64 % PR == 0 && IT % 8 == 0) {
    if (args.nt_out) staged_copy_out<EPI, S, CHF, PR, IT, true>(args, st, mr, nw, lane);
    else staged_copy_out<EPI, S, CHF, PR, IT, false>(args, st, mr, nw, lane);
    return;
  }
  if constexpr (EPI == 4 && !CHECK && 64 % PR == 0 && IT % 2 == 0) {
    if (args.nt_out) staged_side_out<CF, EPI, S, PR, IT, true>(args, st, sd, mr, nw, lane, cs);
    else staged_side_out<CF, EPI, S, PR, IT, false>(args, st, sd, mr, nw, lane, cs);
    return;
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = it * 64 + lane, r = e / PR, p = e % PR;
    const int m = mr + r, n = nw + p * 8;
    const char* row = st + r * S;
    uint4 y;
    if constexpr (F32) {
      const float4 a = *reinterpret_cast<const float4*>(row + p * 32);
      const float4 b = *reinterpret_cast<const float4*>(row + p * 32 + 16);
      float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint32_t w[4] = {sd[it].x, sd[it].y, sd[it].z, sd[it].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float s = bf2f((w[k >> 1] >> (16 * (k & 1))) & 0xffffu);
        if constexpr (EPI != 7) v[k] = EPI == 3 ? v[k] + s : v[k] * s;
      }
      y = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
      if constexpr ((EPI == 4 || EPI == 7) && staged_dbias<CF>()) {  // column sums (fp32, before the bf16 rounding)
        if constexpr (CHECK) {
          const bool ok = m < args.M;
#pragma unroll
          for (int k = 0; k < 8; ++k) cs[k] += (ok && n + k < nlim) ? v[k] : 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) cs[k] += v[k];
        }
      }
    } else {
      y = *reinterpret_cast<const uint4*>(row + p * 16);
    }
    const long off = (long)m * args.ldc + n;
    if constexpr (!CHECK) {
      if (args.nt_out) {  // streamed output far larger than the caches: non-temporal
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4u{y.x, y.y, y.z, y.w},
                                    reinterpret_cast<v4u*>(reinterpret_cast<bf16_t*>(args.C) + off));
        if constexpr (EPI == 2) {
          const uint4 g = *reinterpret_cast<const uint4*>(row + CHF * 16 * S + p * 16);
          __builtin_nontemporal_store(v4u{g.x, g.y, g.z, g.w}, reinterpret_cast<v4u*>(args.aux + off));
        }
      } else {
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(args.C) + off) = y;
        if constexpr (EPI == 2)
          *reinterpret_cast<uint4*>(args.aux + off) = *reinterpret_cast<const uint4*>(row + CHF * 16 * S + p * 16);
      }
    } else if (m < args.M && n < nlim) {
      store8(reinterpret_cast<bf16_t*>(args.C) + off, y, nlim - n);
      if constexpr (EPI == 2)
        store8(args.aux + off, *reinterpret_cast<const uint4*>(row + CHF * 16 * S + p * 16), nlim - n);
    }
  }
}

template <class CF, int EPI, int LDSW>
MG_DEVICE void epilogue_staged(const GemmArgs& args, f32x4 (&acc)[CF::FM][CF::FN], int m0, int n0,
                               int wm, int wn, int wid, int lane, char* smem,
                               unsigned long long* est = nullptr) {
  // EPI 6 / 7: EPI 2 / 4 with GELU' in the fragment order of the W4-256 tiles (frag_aux below).
  // Staged as fp32: EPI 4 (its row-major GELU' side input and the bias gradient's column sums act on
  // the staged values).  The residual (EPI 3) and the fragment-ordered GELU' (EPI 7, whose column sums
  // then run in the fragment layout too) are applied before a bf16 staging: the same fp32 values and
  // the same single rounding, half the LDS passes
  constexpr bool F32 = EPI == 4;
  constexpr int PL = EPI == 2 ? 2 : 1;           // planes: y (+ GELU' for EPI 2)
  constexpr int S = CF::WTN * (F32 ? 4 : 2) + 16;  // row stride: rows 4 banks apart (b64/b128 writes)
  constexpr int CHF = stage_chf(CF::FM, 16 * S * PL, LDSW);  // fragment rows per pass
  constexpr int PR = CF::WTN / 8;                // 8-column pieces per row
  constexpr int IT = CHF * 16 * PR / 64;         // pieces per lane per pass
  static_assert(CHF * 16 * S * PL <= LDSW, "epilogue staging exceeds the wave's LDS share");
  static_assert((CHF * 16 * PR) % 64 == 0, "pieces must fill whole waves");
  char* st = smem + wid * LDSW;
  const int nlim = EPI == 0 ? (int)args.ldc : args.N;
  const int nw = n0 + wn * CF::WTN;
  const int nb = nw + (lane >> 4) * 4;
  const int mw = m0 + wm * CF::WTM;
  uint2 bs[CF::FN];
#pragma unroll
  for (int j = 0; j < CF::FN; ++j) {
    bs[j] = make_uint2(0u, 0u);
    if constexpr (EPI == 1 || EPI == 2 || EPI == 3 || EPI == 6)
      if (args.bias && nb + j * 16 < nlim) bs[j] = *reinterpret_cast<const uint2*>(args.bias + nb + j * 16);
  }
  const bool full = nw + CF::WTN <= nlim && mw + CF::WTM <= args.M;  // wave-uniform: no per-piece checks
  const bf16_t* __restrict__ side = args.aux;
  // EPI 3: residual pieces of row group i + 1 load while row group i is staged (8 bytes per lane and
  // fragment: each wave-instruction reads 32 contiguous bytes of 16 rows, the other fragments of the
  // same lines right behind it)
  constexpr bool ROLL = EPI == 3 || EPI == 7;  // fragment-layout side input, one row group ahead
  uint2 rsd[ROLL ? 2 : 1][ROLL ? CF::FN : 1];
  bf16_t* const frag_aux = (EPI == 6 || EPI == 7)
      ? args.aux + ((long)(m0 / 256) * args.tiles_n + n0 / 256) * 65536 + (long)wid * CF::FM * CF::FN * 256 + lane * 8
      : nullptr;
  auto resid_load = [&](int i, uint2 (&dst)[ROLL ? CF::FN : 1]) __attribute__((always_inline)) {
    if constexpr (EPI == 7) {  // contiguous 1-KiB fragment pairs
#pragma unroll
      for (int j = 0; j < CF::FN; j += 2) {
        const uint4 t = *reinterpret_cast<const uint4*>(frag_aux + (i * CF::FN + j) * 256);
        dst[j] = make_uint2(t.x, t.y);
        dst[j + 1] = make_uint2(t.z, t.w);
      }
    }
    if constexpr (EPI == 3) {
      const int m = mw + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        const int n = nb + j * 16;
        const bf16_t* p = args.resid + (long)m * args.ldc + n;
        if (full) {
          dst[j] = *reinterpret_cast<const uint2*>(p);
        } else if (m < args.M && n < nlim) {
          const uint4 t = load8(p, min(4, nlim - n));
          dst[j] = make_uint2(t.x, t.y);
        } else {
          dst[j] = make_uint2(0u, 0u);
        }
      }
    }
  };
  // (frag_aux: the fragment-ordered GELU' plane -- EPI 6 writes, EPI 7 reads -- per 256 x 256 tile
  // 65536 elements in (wave, i, j / 2, lane, j % 2, 4) order, so each pair of fragments is one fully
  // contiguous 1-KiB wave-instruction of 16-byte lanes from the registers (no LDS staging for that
  // plane) and the fc2 data gradient (same W4-256 tile grid and fragment layout) reads exactly the
  // values its lanes need)
  const uint32_t dkey = EPI == 3 ? rowdrop_key(eff_seed(args.seed, args.sofs)) : 0u;  // dropout key
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // EPI 4 + dbias: this lane's column sums
  float csf[EPI == 7 ? 4 * CF::FN : 1];  // EPI 7: column sums in the fragment layout [j][4]
#pragma unroll
  for (int k = 0; k < (EPI == 7 ? 4 * CF::FN : 1); ++k) csf[k] = 0.f;
  resid_load(0, rsd[0]);
#pragma unroll
  for (int c = 0; c < CF::FM / CHF; ++c) {
    // side inputs of this pass first: their latency hides under the LDS staging
    uint4 sd[F32 ? IT : 1];
    if constexpr (EPI == 4) {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = it * 64 + lane, r = e / PR, n = nw + (e % PR) * 8;
        const int m = mw + c * CHF * 16 + r;
        const bf16_t* p = side + (long)m * args.ldc + n;
        if (full) sd[it] = *reinterpret_cast<const uint4*>(p);
        else sd[it] = m < args.M && n < nlim ? load8(p, nlim - n) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
#pragma unroll
    for (int ii = 0; ii < CHF; ++ii) {
      const int i = c * CHF + ii;
      const int m = mw + i * 16 + (lane & 15);
      char* row = st + (ii * 16 + (lane & 15)) * S;
      if constexpr (ROLL) {
        if (i + 1 < CF::FM) resid_load(i + 1, rsd[(i + 1) & 1]);
      }
      uint32_t gq[4];  // EPI 6: GELU' of fragments j - 1, j (one 16-byte store per pair)
      (void)gq;
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        const int n = nb + j * 16;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (EPI == 1 || EPI == 2 || EPI == 3 || EPI == 6) {
          v[0] += bf2f(bs[j].x & 0xffffu); v[1] += bf2f(bs[j].x >> 16);
          v[2] += bf2f(bs[j].y & 0xffffu); v[3] += bf2f(bs[j].y >> 16);
        }
        const int col = j * 16 + (lane >> 4) * 4;
        if constexpr (EPI == 6) {  // y = GELU(z) staged; GELU'(z) straight to its fragment-ordered plane
          f32x2 y0, y1, g0, g1;
          gelu2(f32x2{v[0], v[1]}, y0, g0);
          gelu2(f32x2{v[2], v[3]}, y1, g1);
          v[0] = y0.x; v[1] = y0.y; v[2] = y1.x; v[3] = y1.y;
          gq[(j & 1) * 2] = pack2(g0.x, g0.y);
          gq[(j & 1) * 2 + 1] = pack2(g1.x, g1.y);
          if (j & 1) {
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(v4u{gq[0], gq[1], gq[2], gq[3]},
                                        reinterpret_cast<v4u*>(frag_aux + (i * CF::FN + j - 1) * 256));
          }
        }
        if constexpr (EPI == 7) {  // x GELU'(z) in the fragment layout (fp32 product, as EPI 4)
          const uint2 gx = rsd[i & 1][j];
          v[0] *= bf2f(gx.x & 0xffffu); v[1] *= bf2f(gx.x >> 16);
          v[2] *= bf2f(gx.y & 0xffffu); v[3] *= bf2f(gx.y >> 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) csf[j * 4 + e] += v[e];  // fp32, before the rounding
        }
        if constexpr (EPI == 2) {  // y = GELU(z); GELU'(z) into the second plane (packed fp32 math)
          f32x2 y0, y1, g0, g1;
          gelu2(f32x2{v[0], v[1]}, y0, g0);
          gelu2(f32x2{v[2], v[3]}, y1, g1);
          v[0] = y0.x; v[1] = y0.y; v[2] = y1.x; v[3] = y1.y;
          *reinterpret_cast<uint2*>(row + CHF * 16 * S + col * 2) =
              make_uint2(pack2(g0.x, g0.y), pack2(g1.x, g1.y));
        }
        if constexpr (EPI == 3) {
          if (args.thr) rowdrop4(v, dkey, m, n, args.N, args.thr, args.scale);  // common.h
          const uint2 rv = rsd[i & 1][j];
          v[0] += bf2f(rv.x & 0xffffu); v[1] += bf2f(rv.x >> 16);
          v[2] += bf2f(rv.y & 0xffffu); v[3] += bf2f(rv.y >> 16);
        }
        if constexpr (F32)
          *reinterpret_cast<float4*>(row + col * 4) = make_float4(v[0], v[1], v[2], v[3]);
        else
          *reinterpret_cast<uint2*>(row + col * 2) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
#ifdef MG_GEMM_EPI_STAMPS
    if (est && c == 0) est[0] = __builtin_amdgcn_s_memtime();  // fragments -> LDS issued
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef MG_GEMM_EPI_STAMPS
    if (est && c == 0) est[1] = __builtin_amdgcn_s_memtime();  // LDS writes landed
#endif
    if (full) staged_rows<CF, EPI, F32, S, CHF, PR, IT, false>(args, st, sd, mw + c * CHF * 16, nw, nlim, lane, cs);
    else staged_rows<CF, EPI, F32, S, CHF, PR, IT, true>(args, st, sd, mw + c * CHF * 16, nw, nlim, lane, cs);
    asm volatile("" ::: "memory");  // the next pass's LDS writes stay behind these reads
#ifdef MG_GEMM_EPI_STAMPS
    if (est) est[2] = __builtin_amdgcn_s_memtime();  // staged reads + global stores issued
#endif
  }
  if constexpr (EPI == 7) {
    if (args.dbias) {
      // the 16 lanes of a column group (lane bits 0-3 = rows) fold by transposing shuffles: lane
      // (r, g) ends with sums 2 r, 2 r + 1 of its 4 FN values ([j][4]: fragment j, column 4 g + e);
      // the NWM row-waves meet in LDS, then one atomic per tile column
      constexpr int NV = 4 * CF::FN;
      static_assert(NV == 32, "fragment-layout fold: 8 fragments per wave-tile row");
#pragma unroll
      for (int M = 8; M >= 1; M >>= 1) {
        const bool hi = lane & M;
        const int C = NV * M / 8;
#pragma unroll
        for (int i2 = 0; i2 < C / 2; ++i2) {
          const float send = hi ? csf[i2] : csf[i2 + C / 2];
          const float keep = hi ? csf[i2 + C / 2] : csf[i2];
          csf[i2] = keep + __shfl_xor(send, M, 64);
        }
      }
      float* red = reinterpret_cast<float*>(smem);  // [NWM][BN], over the staging regions
      __syncthreads();  // every wave's staged reads are done
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int idx = 2 * (lane & 15) + t, j = idx / 4, e = idx % 4;
        red[wm * CF::BN + wn * CF::WTN + 16 * j + 4 * (lane >> 4) + e] = csf[t];
      }
      __syncthreads();
      for (int c = threadIdx.x; c < CF::BN; c += CF::NT) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < CF::NWM; ++r) t += red[r * CF::BN + c];
        if (n0 + c < args.N) atomicAdd(args.dbias + n0 + c, t);
      }
    }
  }
  if constexpr (EPI == 4 && staged_dbias<CF>()) {
    if (args.dbias) {  // kernel argument: uniform over the workgroup
      // lanes sharing a piece index (lane % PR) fold by shuffles, the NWM row-waves through LDS,
      // then one atomic per tile column with 64 contiguous floats per wave-instruction
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int o = PR; o < 64; o <<= 1) cs[k] += __shfl_xor(cs[k], o, 64);
      float* red = reinterpret_cast<float*>(smem);  // [NWM][BN], over the staging regions
      __syncthreads();  // every wave's staged reads are done
      if (lane < PR) {
#pragma unroll
        for (int k = 0; k < 8; ++k) red[wm * CF::BN + wn * CF::WTN + lane * 8 + k] = cs[k];
      }
      __syncthreads();
      for (int c = threadIdx.x; c < CF::BN; c += CF::NT) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < CF::NWM; ++r) t += red[r * CF::BN + c];
        if (n0 + c < args.N) atomicAdd(args.dbias + n0 + c, t);
      }
    }
  }
}

// Shared epilogue: lane holds acc[i][j] = C[m0+wm*WTM+16i+(lane&15)][n0+wn*WTN+16j+4(lane>>4) .. +3].
// LDSW: LDS bytes each wave may use for the staged form (the K-loop's buffers are free by then).
template <class CF, int EPI, bool OUTF32, int LDSW>
MG_DEVICE void epilogue(const GemmArgs& args, f32x4 (&acc)[CF::FM][CF::FN], int m0, int n0, int wm,
                        int wn, int wid, int lane, char* smem, unsigned long long* est = nullptr) {
  if constexpr (!OUTF32) {
    if ((EPI != 4 && EPI != 7) || !args.dbias || staged_dbias<CF>()) {
      epilogue_staged<CF, EPI, LDSW>(args, acc, m0, n0, wm, wn, wid, lane, smem, est);
      return;
    }
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
  // ---- epilogue: lane holds C[m][n..n+3].  Side inputs are loaded a whole row group at a time
  // (bias once per lane; resid / aux / fp32 C for all FN column groups of row m before any use), so a
  // tile pays ~FM load latencies instead of FM x FN serialised round trips.
  const int nlim = (EPI == 0 && !OUTF32) ? (int)args.ldc : args.N;
  const int nb = n0 + wn * CF::WTN + (lane >> 4) * 4;
  const bf16_t* __restrict__ bias = args.bias;
  const uint32_t dkey = EPI == 3 ? rowdrop_key(eff_seed(args.seed, args.sofs)) : 0u;  // dropout key
  uint2 bs[CF::FN];
  float csum[EPI == 4 ? CF::FN : 1][4];  // EPI 4 bias gradient: this lane's column partial sums
#pragma unroll
  for (int j = 0; j < (EPI == 4 ? CF::FN : 1); ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) csum[j][c] = 0.f;
#pragma unroll
  for (int j = 0; j < CF::FN; ++j) {
    bs[j] = make_uint2(0u, 0u);
    if constexpr (EPI == 1 || EPI == 2 || EPI == 3)
      if (bias && nb + j * 16 < nlim) bs[j] = *reinterpret_cast<const uint2*>(bias + nb + j * 16);
  }
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
    const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
    if (m >= args.M) continue;
    const long rowoff = (long)m * args.ldc;
    uint2 side[CF::FN];
    float4 cold[OUTF32 ? CF::FN : 1];
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) {
      const int n = nb + j * 16;
      if (n >= nlim) continue;
      if constexpr (OUTF32) {
        cold[j] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(args.C) + rowoff + n);
      } else if constexpr (EPI == 3) {
        side[j] = *reinterpret_cast<const uint2*>(args.resid + rowoff + n);
      } else if constexpr (EPI == 4) {
        side[j] = *reinterpret_cast<const uint2*>(args.aux + rowoff + n);
      }
    }
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) {
      const int n = nb + j * 16;
      if (n >= nlim) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const long off = rowoff + n;
      if constexpr (OUTF32) {
        float4 c = cold[j];
        c.x += v[0]; c.y += v[1]; c.z += v[2]; c.w += v[3];
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(args.C) + off) = c;
      } else {
        if constexpr (EPI == 1 || EPI == 2 || EPI == 3) {
          v[0] += bf2f(bs[j].x & 0xffffu); v[1] += bf2f(bs[j].x >> 16);
          v[2] += bf2f(bs[j].y & 0xffffu); v[3] += bf2f(bs[j].y >> 16);
        }
        if constexpr (EPI == 2) {  // y = GELU(z); aux <- GELU'(z) for the backward (one multiply there)
          float gd[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sg = gelu_sigmoid(v[r]);
            gd[r] = gelu_grad_from(v[r], sg);
            v[r] *= sg;
          }
          *reinterpret_cast<uint2*>(args.aux + off) = make_uint2(pack2(gd[0], gd[1]), pack2(gd[2], gd[3]));
        }
        if constexpr (EPI == 3) {
          if (args.thr) rowdrop4(v, dkey, m, n, args.N, args.thr, args.scale);  // common.h
          v[0] += bf2f(side[j].x & 0xffffu); v[1] += bf2f(side[j].x >> 16);
          v[2] += bf2f(side[j].y & 0xffffu); v[3] += bf2f(side[j].y >> 16);
        }
        if constexpr (EPI == 4) {  // aux = GELU'(z) stored by the forward's EPI 2
          v[0] *= bf2f(side[j].x & 0xffffu); v[1] *= bf2f(side[j].x >> 16);
          v[2] *= bf2f(side[j].y & 0xffffu); v[3] *= bf2f(side[j].y >> 16);
        }
        const uint2 packed = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if constexpr (EPI == 4) {  // bias gradient of the stored (bf16-rounded) values
          csum[j][0] += bf2f(packed.x & 0xffffu); csum[j][1] += bf2f(packed.x >> 16);
          csum[j][2] += bf2f(packed.y & 0xffffu); csum[j][3] += bf2f(packed.y >> 16);
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(args.C) + off) = packed;
      }
    }
  }
  if constexpr (EPI == 4) {
    if (args.dbias) {
      // sum the 16 rows of each fragment column (lane & 15) by shuffles, the NWM row-waves through
      // LDS, then one full-width atomic pass over the tile's columns (64 contiguous floats per
      // wave-instruction: atomics with a few active lanes each run at a small fraction of that)
      float* cs = reinterpret_cast<float*>(smem);  // [NWM][BN]
#pragma unroll
      for (int j = 0; j < CF::FN; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float t = csum[j][c];
          t += __shfl_xor(t, 1, 64);
          t += __shfl_xor(t, 2, 64);
          t += __shfl_xor(t, 4, 64);
          t += __shfl_xor(t, 8, 64);
          if ((lane & 15) == 0) cs[wm * CF::BN + wn * CF::WTN + j * 16 + (lane >> 4) * 4 + c] = t;
        }
      __syncthreads();
      for (int c = threadIdx.x; c < CF::BN; c += CF::NT) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < CF::NWM; ++r) t += cs[r * CF::BN + c];
        if (n0 + c < args.N) atomicAdd(args.dbias + n0 + c, t);
      }
    }
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
  Stager<AK, CF::BM, CF::NW> sta;
  Stager<BKC, CF::BN, CF::NW> stb;
  sta.init(args.A, args.a_bytes, args.lda, m0, args.a_ext, kbeg, args.ka, kbeg + args.kchunk, wid, lane);
  stb.init(args.B, args.b_bytes, args.ldb, n0, args.b_ext, kbeg, args.kb, kbeg + args.kchunk, wid, lane);
  static_assert(CF::STAGES == 2 && CF::SMEM <= 65536, "two-stage ring with 16-bit stage offsets");
  // prologue: tile 0 in flight
  if (nk > 0) {
    sta.stage(smem, 0);
    stb.stage(smem + CF::A_BYTES, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // two stages: the K-loop unrolled by 2 so each stage's base is a constant that goes into the
  // transposed reads' offset fields (the W4 slot unroll, same reasoning); per K-tile: DMA of tile
  // kt+1 into the other stage, the two k32 steps, then tile kt+1 landed (this wave's DMA) and every
  // wave's LDS reads of stage kt retired before the barrier
  auto ktile2 = [&](int kt, auto st_c) __attribute__((always_inline)) {
    constexpr int ST = decltype(st_c)::value;
    constexpr int OA = ST * CF::STAGE, OB = OA + CF::A_BYTES, ON = (ST ^ 1) * CF::STAGE;
    const int kn = kt + 1;
    if (kn < nk) {  // its stage was last read in iteration kt-1: free since that barrier
      sta.stage(smem + ON, kn);
      stb.stage(smem + ON + CF::A_BYTES, kn);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[CF::FM], fb[CF::FN];
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
        fa[i] = ks ? frag_k<AK, 1, 16384, OA>(smem, wm * CF::FM + i, lane)
                   : frag_k<AK, 0, 16384, OA>(smem, wm * CF::FM + i, lane);
#pragma unroll
      for (int j = 0; j < CF::FN; ++j)
        fb[j] = ks ? frag_k<BKC, 1, 16384, OB>(smem, wn * CF::FN + j, lane)
                   : frag_k<BKC, 0, 16384, OB>(smem, wn * CF::FN + j, lane);
      if constexpr (!AK || !BKC) {
        lds_ready(fa);
        lds_ready(fb, false);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    ktile2(kt, std::integral_constant<int, 0>{});
    ktile2(kt + 1, std::integral_constant<int, 1>{});
  }
  if (kt < nk) ktile2(kt, std::integral_constant<int, 0>{});

  epilogue<CF, EPI, OUTF32, CF::SMEM / CF::NW>(args, acc, m0, n0, wm, wn, wid, lane, smem);
}

// Split-K for the fp32-accumulate (weight-gradient) layout: pick the split that minimises
// rounds x per-block work, where rounds = ceil(blocks / concurrent slots) and per-block work =
// its K-tiles + ~2 tiles of prologue/epilogue (the atomic write-back).  A naive "fill the chip"
// split leaves a mostly idle second round (e.g. 144 tiles x 4 = 576 blocks on 512 slots).
static int choose_split(int tiles, int slots, int nkt, int ovh, int spmin = 1, long* cost = nullptr) {
  int best = spmin;
  long bc = -1;
  const int maxsp = std::max(spmin, std::min(32, nkt / 4));
  for (int sp = spmin; sp <= maxsp; ++sp) {
    const long rounds = ((long)tiles * sp + slots - 1) / slots;
    const long c = rounds * (cdiv(nkt, sp) + ovh);
    if (bc < 0 || c * 20 < bc * 19) {  // a further split must save >= 5%
      bc = c;
      best = sp;
    }
  }
  if (cost) *cost = bc;
  return best;
}

// ovh: per-block prologue + atomic write-back in K-tile units (grows with the tile area)
static void set_split(GemmArgs& a, int slots, int ovh) {
  const int nkt = cdiv(a.K, BK);
  // a split's K range of an m/n-contiguous operand (k rows of ld elements) must stay inside one
  // buffer descriptor (< 4 GiB from the split's origin): the LM head's weight gradient at 131k
  // tokens reads 13 GB of logits gradients in one launch (6 splits: half the fp32 atomic bytes of
  // the four row-chunked launches of 3 splits each, and no per-launch round quantisation)
  const uint64_t row_bytes = (uint64_t)std::max(a.lda, a.ldb) * 2;
  int spmin = 1;
  while (spmin < nkt && (uint64_t)cdiv(nkt, spmin) * BK * row_bytes >= 0xF0000000ull) ++spmin;
  const int sp = choose_split(a.tiles_m * a.tiles_n, slots, nkt, ovh, spmin);
  a.kchunk = cdiv(nkt, sp) * BK;
  a.splits = cdiv(a.K, a.kchunk);
}

// ============================================================================================
// 4-wave 256x256 kernel ("W4"): one wave per SIMD, 128x128 wave tile (256 accumulator registers,
// 512-register budget), the structure that keeps MFMA busy without a partner wave.
//
// Per K-tile kt (BK = 64 = two k32 steps, the T256 images; A in a 2-slot LDS ring, slot kt & 1,
// B in a 3-slot ring, slot kt % 3):
//   phase A: 64 MFMAs on the k32 step-0 fragments; step-1 fragments of tile kt read; LDS-DMA of
//            tile kt+2's B into B slot (kt+2) % 3 (it held tile kt-1, fully read before the
//            previous K-tile's barrier)
//   s_waitcnt vmcnt(B pieces) lgkmcnt(0) + barrier   (tile kt+1 landed; A slot kt & 1 fully read)
//   phase B: 64 MFMAs on the step-1 fragments; step-0 fragments of tile kt+1 read; LDS-DMA of
//            tile kt+2's A into A slot kt & 1
// One barrier per K-tile, and the K-tile's DMA (64 KiB per CU, ~1k cycles of the CU's ~64 B/clk
// LDS-DMA path) is split evenly over both phases, one piece per 8 MFMAs: issued in one phase it
// out-ran the DMA path and stalled the in-order MFMA stream behind it (tools/gemm_stamps.hip:
// phase B 1.94k cycles with the pieces bunched, 1.47k spread over phase B, phase A 1.08k).
// The third B slot replaces the old DMA sink: DMA past the last K-tile re-reads tile 0 into
// slots nobody reads again, so every K-tile waits with the same counts.
// MFMA with the accumulator pinned to AGPRs ("+a"): with 256 accumulator registers the compiler's
// own allocation shuffles them between AGPRs and VGPRs every K-step.  volatile + "memory" keeps
// program order between the MFMAs and the LDS reads / DMA pieces placed between them: one wave per
// SIMD issues in order, so a burst of loads would stall its own MFMA stream.
MG_DEVICE void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b) : "memory");
}

// BN = 256 (128x128 wave tiles) or 192 (128x96: 2 rounds instead of 1.5 for N = 768 on 256 CUs;
// k-contiguous B only -- the m/n-contiguous half-images are 128 columns wide)
template <int BN>
struct W4 {
  static constexpr int FN = BN / 32;                  // 16-col fragments per wave (2 x 2 waves)
  static constexpr int A_SLOT = 32768;                // 256 x 64 bf16
  static constexpr int B_SLOT = BN * 128;             // BN x 64 bf16
  static constexpr int B_RING = 2 * A_SLOT;           // [A0][A1][B0][B1][B2]
  static constexpr int SMEM = 2 * A_SLOT + 3 * B_SLOT;  // 160 KiB at BN = 256
  static constexpr int NR = 8 + FN;                   // fragment reads per phase
  static constexpr int PA = 8, PB = FN;               // DMA pieces per wave per K-tile (A, B)
};

// DMA piece issued after MFMA q of a phase (or -1): NR pieces spread evenly over the NQ MFMAs.
template <int NQ, int NR>
MG_DEVICE constexpr int w4_piece_at(int q) {
  for (int r = 0; r < NR; ++r)
    if (r * NQ / NR == q) return r;
  return -1;
}

// K-tile visited s-th (tail_first: the partial last K-tile, then 0, 1, ...)
MG_DEVICE int w4_tile(int s, int nk, bool tail_first) { return tail_first ? (s == 0 ? nk - 1 : s - 1) : s; }

// the K-loop's final MFMA with the wait states its result needs before any VALU / scratch read
// (hipcc cannot see the latency of an asm MFMA; whatever it places after the loop -- epilogue reads,
// spill stores -- must not start inside that window)
MG_DEVICE void mfma_acc_last(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7" : "+a"(acc) : "v"(a), "v"(b) : "memory");
}


template <int BN, bool AK, bool BKC, int EPI, bool OUTF32>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const GemmArgs args) {
  static_assert(BN == 256 || BKC, "W4 with BN != 256 needs a k-contiguous B operand");
  using CF = Cfg<256, BN, 2, 2>;
  using WK = W4<BN>;
  constexpr int FN = WK::FN, NR = WK::NR, NQ = 8 * FN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int nblk = args.tiles_m * args.tiles_n * args.splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wgs = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int ntiles = args.tiles_m * args.tiles_n;
  const int split = wgs / ntiles;
  const int wg = wgs % ntiles;
  const int group = GROUP_M * args.tiles_n;
  const int first_m = (wg / group) * GROUP_M;
  const int gm = min(args.tiles_m - first_m, GROUP_M);
  const int m0 = (first_m + (wg % group) % gm) * 256;
  const int n0 = ((wg % group) / gm) * BN;

#ifdef MG_GEMM_STAMPS
  // diagnostic builds: [0..5] segments of K-tile MG_GEMM_STAMPS (phase A issue | wait | barrier |
  // phase B | fragment wait), [6..9] kernel start | main loop start | main loop end | end
  unsigned long long st[10];
#define W4_STAMP(k) st[k] = __builtin_amdgcn_s_memtime()
#define W4_KSTAMP(k) if (kt == MG_GEMM_STAMPS) st[k] = __builtin_amdgcn_s_memtime()
#else
#define W4_STAMP(k)
#define W4_KSTAMP(k)
#endif
  W4_STAMP(6);
  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kbeg = split * args.kchunk;
  const int nk = (min(args.K, kbeg + args.kchunk) - kbeg + BK - 1) / BK;
  // m/n-contiguous operands (the data and weight gradients): the ring's slots interleaved inside
  // each 128-column half-image (16 KiB per slot and half), so that with the K-loop unrolled over
  // the slot pattern every transposed read's slot offset is a constant in its offset field
  // (every layout: the all-k-contiguous forward gained +0.4 % of the step too, its slot bases then
  // fold into the reads' offsets; profiles/round4_w4_nt_unroll_ab.txt)
  constexpr int AS = AK ? WK::A_SLOT : 16384, AHS = 2 * 16384;  // A: slot / half-image strides
  constexpr int BS = BKC ? WK::B_SLOT : 16384, BHS = 3 * 16384;  // B: 3 slots
  Stager<AK, 256, 4, AHS> sta;
  Stager<BKC, BN, 4, BHS> stb;
  sta.init(args.A, args.a_bytes, args.lda, m0, args.a_ext, kbeg, args.ka, kbeg + args.kchunk, wid, lane);
  stb.init(args.B, args.b_bytes, args.ldb, n0, args.b_ext, kbeg, args.kb, kbeg + args.kchunk, wid, lane);
  // K-tile visiting order: a partial last K-tile (K % 64 != 0; W4 layouts have ka = kb = K and
  // split-K chunks of whole tiles, so it is the only tile needing per-lane k checks) goes first,
  // staged in the prologue, so the main loop's DMA pieces carry no check (a v_cndmask each)
  const bool tail_first = (sta.klim % BK) != 0;
  char* const sB = smem + WK::B_RING;
  sta.stage(smem, w4_tile(0, nk, tail_first));
  stb.stage(sB, w4_tile(0, nk, tail_first));
  if (nk > 1) {
    sta.stage(smem + AS, w4_tile(1, nk, tail_first));
    stb.stage(sB + BS, w4_tile(1, nk, tail_first));
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WK::PA + WK::PB) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  bf16x8 fa0[8], fb0[FN], fa1[8], fb1[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb0[j] = frag_k<BKC, 0, BHS>(sB, wn * FN + j, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = frag_k<AK, 0, AHS>(smem, wm * 8 + i, lane);
  lds_ready(fa0);
  lds_ready(fb0, false);
  W4_STAMP(7);

  // One K-tile with compile-time ring slots SA (A, kt & 1) and SB (B, kt % 3), so every slot base
  // is a constant in the LDS reads' offset fields and the K-loop below is unrolled over the 6-tile
  // slot pattern
  auto ktile = [&](int kt, auto sa_c, auto sb_c) __attribute__((always_inline)) {
    constexpr int SA = decltype(sa_c)::value, SB = decltype(sb_c)::value;
    constexpr int OA = SA * AS, OA1 = (SA ^ 1) * AS;
    constexpr int OB = SB * BS, OB1 = ((SB + 1) % 3) * BS, OB2 = ((SB + 2) % 3) * BS;
    W4_KSTAMP(0);
    const int t2 = kt + 2;
    // past the end: re-read a tile into a slot nobody reads (every K-tile waits with the same counts)
    const int tt = w4_tile(t2 < nk ? t2 : 1, nk, tail_first);
    // phase A: k32 step 0 of tile kt; step-1 fragments read between the MFMAs (one per 2, B first:
    // the next phase's first FN MFMAs use fa[0] with every fb[j]); B of tile kt+2 by DMA into B
    // slot (kt+2) % 3
    {
      const __amdgpu_buffer_rsrc_t rb = stb.rsrc(tt);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int i = q / FN, j = q % FN;
        mfma_acc(acc[i][j], fb0[j], fa0[i]);
        if ((q & 1) == 0 && q < 2 * NR) {
          const int r = q >> 1;
          if (r < FN) fb1[r] = frag_k<BKC, 1, BHS, OB>(sB, wn * FN + r, lane);
          else fa1[r - FN] = frag_k<AK, 1, AHS, OA>(smem, wm * 8 + r - FN, lane);
        }
        if (w4_piece_at<NQ, WK::PB>(q) >= 0) stb.piece(sB + OB2, rb, tt, w4_piece_at<NQ, WK::PB>(q), false);
      }
    }
    // tile kt+1 landed (this wave's DMA older than the B pieces just issued), every wave done
    // reading A slot kt & 1
    W4_KSTAMP(1);
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WK::PB) : "memory");
    lds_ready(fa1, false);
    lds_ready(fb1, false);
    W4_KSTAMP(2);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    W4_KSTAMP(3);
    // phase B: k32 step 1 of tile kt; A of tile kt+2 by DMA into A slot kt & 1; step-0 fragments
    // of tile kt+1 between the MFMAs, B first, early in the phase so they have ~3/4 of it to land
    // before the next phase A needs them
    {
      const __amdgpu_buffer_rsrc_t ra = sta.rsrc(tt);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int i = q / FN, j = q % FN;
        // every K-tile's final MFMA carries the wait states (a branch on "last K-tile" makes hipcc
        // duplicate the accumulator into other AGPRs; 16 cycles per 2048 is cheaper than that)
        if (q == NQ - 1) mfma_acc_last(acc[i][j], fb1[j], fa1[i]);
        else mfma_acc(acc[i][j], fb1[j], fa1[i]);
        if (w4_piece_at<NQ, WK::PA>(q) >= 0) sta.piece(smem + OA, ra, tt, w4_piece_at<NQ, WK::PA>(q), false);
        if (q < 2 * NR && (q & 1) == 1) {
          const int r = q >> 1;
          if (r < FN) fb0[r] = frag_k<BKC, 0, BHS, OB1>(sB, wn * FN + r, lane);
          else fa0[r - FN] = frag_k<AK, 0, AHS, OA1>(smem, wm * 8 + r - FN, lane);
        }
      }
    }
    W4_KSTAMP(4);
    lds_ready(fa0);  // read early in phase B: long landed, the wait is free
    lds_ready(fb0, false);
    W4_KSTAMP(5);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;

  // slot pattern of K-tiles 6n .. 6n + 5: (A, B) = (0,0) (1,1) (0,2) (1,0) (0,1) (1,2)
  int kt = 0;
  for (; kt + 6 <= nk; kt += 6) {
    ktile(kt, I0{}, I0{});
    ktile(kt + 1, I1{}, I1{});
    ktile(kt + 2, I0{}, I2{});
    ktile(kt + 3, I1{}, I0{});
    ktile(kt + 4, I0{}, I1{});
    ktile(kt + 5, I1{}, I2{});
  }
  if (kt < nk) ktile(kt, I0{}, I0{});
  if (kt + 1 < nk) ktile(kt + 1, I1{}, I1{});
  if (kt + 2 < nk) ktile(kt + 2, I0{}, I2{});
  if (kt + 3 < nk) ktile(kt + 3, I1{}, I0{});
  if (kt + 4 < nk) ktile(kt + 4, I0{}, I1{});
  W4_STAMP(8);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
#ifdef MG_GEMM_EPI_STAMPS
  epilogue<CF, EPI, OUTF32, WK::SMEM / 4>(args, acc, m0, n0, wm, wn, wid, lane, smem, st);
#else
  epilogue<CF, EPI, OUTF32, WK::SMEM / 4>(args, acc, m0, n0, wm, wn, wid, lane, smem);
#endif
#ifdef MG_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores drained
  W4_STAMP(9);
  if (args.dbg && lane == 0)
    for (int k = 0; k < 10; ++k) args.dbg[((long)blockIdx.x * 8 + wid) * 24 + k] = st[k];
#endif
#undef W4_STAMP
#undef W4_KSTAMP
}

template <int BN, bool AK, bool BKC, int EPI, bool OUTF32>
void launch_w4(GemmArgs a, hipStream_t stream) {
  if constexpr (BN != 256 && !BKC) {
    launch_w4<256, AK, BKC, EPI, OUTF32>(a, stream);
  } else {
    a.tiles_m = cdiv(a.M, 256);
    a.tiles_n = cdiv(a.N, BN);
    a.splits = 1;
    a.kchunk = cdiv(a.K, BK) * BK;
    if (OUTF32) set_split(a, 256, 6);
    const int tiles = a.tiles_m * a.tiles_n * a.splits;
    const int grid = tiles;
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute((const void*)gemm_w4_kernel<BN, AK, BKC, EPI, OUTF32>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, W4<BN>::SMEM);
      attr_set = true;
    }
    gemm_w4_kernel<BN, AK, BKC, EPI, OUTF32><<<grid, 256, W4<BN>::SMEM, stream>>>(a);
  }
}

template <class CF, bool AK, bool BKC, int EPI, bool OUTF32>
void launch(GemmArgs a, hipStream_t stream) {
  a.tiles_m = cdiv(a.M, CF::BM);
  a.tiles_n = cdiv(a.N, CF::BN);
  a.splits = 1;
  a.kchunk = cdiv(a.K, BK) * BK;
  if (OUTF32) set_split(a, 256 * (CF::SMEM <= 80 * 1024 ? 2 : 1), 2 + CF::BM * CF::BN / 16384);
  const int grid = a.tiles_m * a.tiles_n * a.splits;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_kernel<CF, AK, BKC, EPI, OUTF32>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, CF::SMEM);
    attr_set = true;
  }
  gemm_kernel<CF, AK, BKC, EPI, OUTF32><<<grid, CF::NT, CF::SMEM, stream>>>(a);
}

// Tile config per shape and layout (bench/bench_gemm.py, bench_wgrad.py, dgrad_nn_vs_nt.py):
//   forward (NT):  W4 (256x256, or 256x192 where that quantises better onto the 256 CUs) once there
//                  is at least one full round of 256^2 tiles; T128 below that (gpt-mini)
//   dgrad (NN):    W4 from one round of 256^2 tiles up, T128 below
//   wgrad (TN):    W4 or T128 through the split-K cost model (below)
int pick_config(int M, int N, int K, int layout) {
  if (g_variant) return g_variant;
  const long tm = cdiv(M, 256);
  const long t256 = tm * cdiv(N, 256);
  if (layout == 0) {
    if (t256 < 256) return 1;
    // (the LM head's data gradient, N = 768, K = 50304, went to the 128x96 wave tile until round 6:
    // with interleaved timing the 256-wide tile is 2.1-2.4 % faster at 65k and 131k tokens,
    // profiles/round6_gemm_vs_hipblaslt_*.jsonl)
    // W4 width: fewer (rounds x tile width) on the 256 CUs wins; the 96-wide wave tile costs ~8 %
    // more per FLOP (more LDS reads per MFMA), so it must save more than that
    const long r256 = (t256 + 255) / 256 * 256, r192 = (tm * cdiv(N, 192) + 255) / 256 * 192;
    return r192 * 108 < r256 * 100 ? 6 : 5;
  }
  // dgrad (NN, the weight read in place through the transposing LDS reads): W4 at every block
  // shape (bench/dgrad_nn_vs_nt.py, M = 65536, W4 / the deleted ping-pong: proj 84 / 97 us, fc 251 / 290, qkv 182 / 210,
  // fc2 + GELU' 344 / 362), and faster than NT against a transposed weight copy
  if (layout == 1) return t256 >= 256 ? 5 : 1;
  // tiny outputs (gpt-mini) on T128; from 512 x 512 up the split-K cost model decides: the 768 x 768
  // attention-projection gradient at 131k tokens runs 164 us on W4 vs 181 on T128 (bench_wgrad.py)
  if ((long)M * N < (1L << 18)) return 1;
  // wgrad: W4 (256^2 tiles, one block per CU, split-K over 256 slots) unless T128 (128^2, two
  // blocks per CU, 512 slots) quantises so much better that it pays for its ~15 % lower per-CU
  // rate.  Both sides through the split-K cost model (rounds x (K-tiles per block + overhead)); a
  // T128 K-tile is a quarter of the work at 2 blocks per CU and ~0.77 of W4's rate since W4's
  // TN main loop lost its address VALU (round 4): 0.65 W4 K-tiles (was 0.59 at 0.85).
  // bench_wgrad.py (profiles/round4_wgrad_pick_xl.txt): gpt2-xl at 16k tokens qkv 257 vs 296 us
  // and attention projection 102 vs 108 on T128, at 32k tokens 493 vs 523 and 168 vs 173 on W4
  // (xl B = 32 step +0.7 %); every GPT-2 (131k tokens) and LM-head shape on W4.
  const int nkt = cdiv(K, BK);
  long c4 = 0, c1 = 0;
  choose_split((int)t256, 256, nkt, 6, 1, &c4);
  choose_split(cdiv(M, 128) * cdiv(N, 128), 512, nkt, 3, 1, &c1);
  return c1 * 65 < c4 * 100 ? 1 : 5;
}

template <bool AK, bool BKC, int EPI, bool OUTF32>
void dispatch(const GemmArgs& a, hipStream_t stream) {
  const int layout = OUTF32 ? 2 : (BKC ? 0 : 1);
  switch (pick_config(a.M, a.N, a.K, layout)) {
    case 5: launch_w4<256, AK, BKC, EPI, OUTF32>(a, stream); break;
    case 6: launch_w4<192, AK, BKC, EPI, OUTF32>(a, stream); break;
    default: launch<T128, AK, BKC, EPI, OUTF32>(a, stream); break;
  }
}

}  // namespace

namespace mg {

int gemm_pick(int M, int N, int K, int layout) { return pick_config(M, N, K, layout); }

void gemm_set_variant(int v) {
  if (v != 0 && v != 1 && v != 5 && v != 6) throw std::invalid_argument("gemm_set_variant: 0 (auto), 1 (T128), 5 (W4), 6 (W4 BN=192)");
  g_variant = v;
}
void gemm_set_debug_buffer(unsigned long long* p) { g_dbg = p; }
int gemm_get_variant() { return g_variant; }

// layout: 0 = NT (fwd), 1 = NN (dgrad), 2 = TN (wgrad, fp32 accumulate into C)
void gemm(int layout, int epi, const bf16_t* A, const bf16_t* B, void* C, long lda, long ldb,
          long ldc, int M, int N, int K, int a_ext, int b_ext, int ka, int kb, const bf16_t* bias,
          bf16_t* aux, const bf16_t* resid, float p, uint64_t seed, hipStream_t stream,
          size_t a_bytes, size_t b_bytes, float* dbias) {
  GemmArgs a;
  a.dbias = dbias;
  a.a_bytes = a_bytes;  // full sizes: each block's descriptor starts at its own tile / split origin
  a.b_bytes = b_bytes;
  a.A = A; a.B = B; a.C = C; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K; a.a_ext = a_ext; a.b_ext = b_ext; a.ka = ka; a.kb = kb;
  a.bias = bias; a.aux = aux; a.resid = resid; a.seed = seed; a.sofs = graph_seed_ofs();
  a.thr = dropout_threshold16(p);  // EPI 3 residual dropout: 16-bit row-block mask (common.h)
  a.scale = dropout_scale16(a.thr);
  a.tiles_m = a.tiles_n = a.splits = 1;
  a.kchunk = K;
  a.dbg = g_dbg;
  // bf16 outputs are written non-temporally: they are consumed by a later kernel, and keeping them
  // out of L2 / MALL leaves those to the GEMM operands (one-box A/B at B = 64: LM head forward
  // 5.07 -> 4.51 ms; step +1.3 % with every output > 256 MB, +0.5 % more with all of them)
  a.nt_out = 1;
  if (layout == 0) {
    if (epi == 0) dispatch<true, true, 0, false>(a, stream);
    else if (epi == 1) dispatch<true, true, 1, false>(a, stream);
    else if (epi == 2) dispatch<true, true, 2, false>(a, stream);
    else if (epi == 3) dispatch<true, true, 3, false>(a, stream);
    else if (epi == 6) launch_w4<256, true, true, 6, false>(a, stream);  // fragment-ordered GELU': W4-256 only
    else dispatch<true, true, 4, false>(a, stream);  // dgrad as NT against a transposed weight
  } else if (layout == 1) {
    if (epi == 4) dispatch<true, false, 4, false>(a, stream);
    else if (epi == 7) launch_w4<256, true, false, 7, false>(a, stream);
    else dispatch<true, false, 0, false>(a, stream);
  } else {
    dispatch<false, false, 0, true>(a, stream);
  }
}

}  // namespace mg
