// Causal flash attention forward for training on gfx950 (CDNA4, MI355X): the dropout keep-bit
// generator and the forward kernel.  (Backward: attention_train.hip; decode: attention.hip.)
//
//
// Replaces the reference's nn.MultiheadAttention math path
// (/root/reference/mingpt/model.py:147-165: in-proj split, q*scale, baddbmm with the [T,T] mask,
// softmax, dropout, bmm PV, plus the discarded head-averaged weights) with a true causal kernel
// that never materialises [T, T] (fixes D4: the reference's additive 0/1 mask was not causal).
//
// Head dims: any multiple of 8 up to 128.  The kernels are instantiated per number of 16-column
// MFMA k-steps (NKS = ceil(hd / 16) rounded to {1, 2, 3, 4, 6, 8}); columns past hd are zero in
// the LDS images and the Q fragments, so they add nothing.  LDS images hold 64 columns per row;
// hd > 64 uses two 64-column halves (attn_common.h).
//
// Dropout on the attention probabilities (the reference's MHA dropout, model.py:150): the keep
// bits are generated up front by attn_dropmask_kernel -- one u32 per (b, h, 64-key tile half,
// query) -- and read by both passes, so the forward's inner loop carries no hashing (at hd = 64
// the forward is VALU-bound: the hash was ~40 % of its vector instructions).
//
// Forward (FA2 structure, MI355X mapping):
//  * workgroup = 4 waves = 128 queries of one (b, h); each wave owns 32 queries.
//  * Q fragments live in VGPRs for the whole kernel, pre-multiplied by log2(e)/sqrt(hd): S comes
//    out of the MFMA in the log2 domain and p = exp2(S - m) costs one subtract per score.
//  * K/V tiles of 64 keys are staged through LDS (double buffer; tile t+1's global loads are in
//    flight during tile t's MFMAs; per-thread addresses are computed once).
//  * S^T = K Q^T with v_mfma_f32_32x32x16_bf16 ("swapped" operands): the query is on the lane, so
//    the softmax row statistics are lane-local; the two 32-key halves of a row meet through one
//    v_permlane32_swap (max) and the row sum is combined only once, after the last tile.
//  * the online-softmax rescale is lazy: a row's running max moves only when a score exceeds it
//    by more than 8 (log2 units; p <= 256 in between), which after the first tile is rare.
//  * P is converted to bf16 in registers and used directly as the B operand of O^T = V^T P^T;
//    V^T fragments come from LDS with ds_read_b64_tr_b16 in the matching permuted key order.
//  * heaviest (last) query blocks are launched first; fully-masked K tiles are skipped per wave.
#include <type_traits>

#include "attn_common.h"
#include "kernels.h"

using namespace mg;
using namespace mg::attn;

namespace {

#ifndef MG_FWD_PAIR
#define MG_FWD_PAIR 1  // forward workgroup = two query blocks (heaviest + lightest), XCD-grouped
#endif

// ------------------------------------------------------------------------------- dropout bits
// Keep bits (keep iff a 16-bit uniform >= thr) as "row words": word (bh, j, q), j = 2 * tile + h, covers
// the 32 scores one forward lane holds for query q in 64-key tile `tile`, half h: value
// e = 16 * sub + r  <->  key 64 * tile + 32 * sub + 4 * h + (r & 3) + 8 * (r >> 2), at bit
// drop_bit(e) = 16 (e & 1) + (e >> 1) (attn_common.h): the two scores of packed pair
// j = e >> 1 (one bf16x2 word of the P operand) sit at bits j and 16 + j, so one shift and one
// packed 16-bit arithmetic shift make the pair's 32-bit keep mask (attn_fwd_pipe_kernel).  Stored
// [bh][j][q]: lanes of consecutive queries read consecutive words in both passes; the backward
// tests a per-lane bit.  Randomness: one lowbias32 mix of the word index and seed, then xorshift32
// steps -- shifts and xors only (32-bit integer multiplies are quarter rate), 16 bits a decision.
//   Tried and removed: the same bits also transposed (32 ballots per wave) into per-register SGPR
// lane masks so the forward drops a score with ONE v_cndmask_b32: at B = 128 the mask kernel went
// 106 -> 277 us and the forward gained ~20 us (scalar loads, SGPR spills).
__global__ __launch_bounds__(256) void attn_dropmask_kernel(uint32_t* __restrict__ dmask,
                                                            int BH, int T, int ntw, int ng, int nt,
                                                            uint64_t seed,
                                                            const uint64_t* __restrict__ sofs,
                                                            uint32_t thr) {
  // grid (BH, ceil(ng / 4)); wave -> query group G (32 queries x 2 halves on its 64 lanes), tiles
  // up to the group's diagonal (the forward and backward read no word past it); 32-bit index math
  const int bh = blockIdx.x;
  const int G = blockIdx.y * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (G >= ng) return;
  const int lane = threadIdx.x & 63;
  const int q = 32 * G + (lane & 31), h = lane >> 5;
  const uint64_t sd = eff_seed(seed, sofs);
  const uint32_t key = (uint32_t)sd ^ mix32((uint32_t)(sd >> 32) + 0x9E3779B9u);
  // exact 16-bit decisions (keep iff a 16-bit uniform u >= thr, thr = round(65536 p) in [1, 65535]):
  // both halves at once, min(sat(u - (thr - 1)), 1) = [u >= thr] (v_pk_sub_u16 clamp, v_pk_min_u16)
  const uint32_t tm1 = (thr - 1u) * 0x00010001u, one = 0x00010001u;
  const int tmax = min(nt - 1, G >> 1);
  for (int t = 0; t <= tmax; ++t) {
    const int j = 2 * t + h;
    uint32_t bits = 0;
    if (q < T) {
      const uint32_t i = (uint32_t)((bh * ntw + j) * T + q);  // the word's index (wraps past 2^32: fine)
      uint32_t x = mix32(i ^ key) | 1u;
#pragma unroll
      for (int w = 0; w < 16; ++w) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        // the two decisions land at bits w, 16 + w (values e = 2w, 2w + 1): drop_bit(e)
        // (asm: the builtins became two compares and selects per half)
        uint32_t k;
        asm("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, %3" : "=&v"(k) : "v"(x), "v"(tm1), "v"(one));
        bits |= k << w;
      }
      dmask[((long)bh * ntw + j) * T + q] = bits;
    }
  }
}


// One 64-key tile for one wave's 32 queries: S'^T = K Q^T - m (the running max m rides in as the
// MFMA's C operand), p = exp2(S'), O^T += V^T (Z P)^T.  There is no per-tile row max: m moves
// only when a tile's partial row sum leaves [lo, 2^60] (lo = 2^-60 on a block's first tile, where
// m starts at 0, else 0) -- then the tile is recomputed against its row max (regrow; rare: bf16 P
// and the fp32 O / l accumulators hold p up to 2^60 exactly as well as p near 1).
template <int NKS, bool MASK, bool DROP>
MG_DEVICE void fwd_tile(const char* sk, const char* sv, const int (&ko)[NKS], const bf16x8 (&qf)[NKS],
                        f32x16 (&o)[(NKS + 1) / 2], f32x16& negm, float& m, float& l, bool first,
                        uint32_t kw, int lim, int ta0, int tb0, int ta1, int tb1) {
  constexpr int NO = (NKS + 1) / 2;
  constexpr int HALF = 64 * ROWB;
  f32x16 s[2];
  auto scores = [&](int lim) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk + sub * 32 * ROWB, ko[0]), qf[0], negm, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < NKS; ++ks)
        s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk + sub * 32 * ROWB, ko[ks]), qf[ks],
                                                         s[sub], 0, 0, 0);
    }
    if constexpr (MASK) {  // key = k0 + c(sub, r) + 4 h32, c a constant: one compare per score
      // lim made opaque here: the compares cannot be hoisted above the MFMAs (32 compare
      // results held in SGPR pairs meanwhile were most of this kernel's scalar pressure)
      asm volatile("" : "+v"(lim));
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[sub][r] = (sub * 32 + (r & 3) + 8 * (r >> 2) > lim) ? kNegBig : s[sub][r];
    }
  };
  auto expsum = [&]() {
    float rs = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(s[sub][r]);
        rs += p;
        s[sub][r] = p;
      }
    return rs;
  };
  scores(lim);
  float rs = expsum();
  const float lo = first ? 8.673617379884035e-19f : 0.f;  // 2^-60
  if (__builtin_expect(__any(!(rs <= 1.152921504606847e18f && rs >= lo)), 0)) {  // 2^60; inf / nan
    // recompute S' (K is still in LDS) instead of keeping it live; an opaque copy of lim keeps
    // the compiler from holding the first pass's 32 mask compares (64 SGPRs) for this one
    int lim2 = lim;
    asm volatile("" : "+v"(lim2));
    scores(lim2);
    float mx = s[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[1][r]);
    mx = max_xor32(mx);
    // a block's first tile may move m down as well (nothing accumulated yet); later tiles up only
    const float d = first ? mx : fmaxf(mx, 0.f);
    const float alpha = first ? 1.f : fexp2(-d);
    l *= alpha;
#pragma unroll
    for (int n = 0; n < NO; ++n) o[n] *= alpha;
    m += d;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = -m;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[sub][r] -= d;
    rs = expsum();
  }
  l += rs;
  // dropout for O only (l sums the undropped P); the keep scale is applied to O at the end
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    if constexpr (DROP) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int bit = drop_bit(16 * sub + r);
        const int keep = (int)(kw << (31 - bit)) >> 31;  // sign-extended bit: one v_bfe_i32
        s[sub][r] = __int_as_float(__float_as_int(s[sub][r]) & keep);
      }
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 pf = pack_frag(s[sub], st);
      const int rb = (sub * 32 + 16 * st) * ROWB;  // 16-row aligned: an immediate
#pragma unroll
      for (int n = 0; n < NO; ++n) {
        const char* vb = sv + (n >> 1) * HALF + rb;
        o[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            (n & 1) ? lds_tr_at(vb, ta1, tb1) : lds_tr_at(vb, ta0, tb0), pf, o[n], 0, 0, 0);
      }
    }
  }
}

// Forward, FA2 structure mapped onto MI355X:
//  * workgroup = 4 waves; a query block = 128 queries of one (b, h), each wave 32 of them; the
//    workgroup runs TWO query blocks of its (b, h) back to back, the i-th heaviest and the i-th
//    lightest (causal work (nqb - 1 - i) + i + 2 tiles pairs: every workgroup the same), and the
//    K/V tile stream continues across the seam (the second block's first tile is prefetched
//    during the first block's last).
//  * XCD-aware grid: the workgroups of one (b, h) are dispatched 8 apart, i.e. onto one XCD
//    under round-robin placement, within one dispatch window: they share K/V through that XCD's
//    L2 instead of each pulling them from HBM (speed only; correctness never depends on it).
//  * Q fragments live in VGPRs, pre-multiplied by log2(e)/sqrt(hd): S comes out of the MFMA in
//    the log2 domain; the running max enters as the MFMA's C operand, so p = exp2(S') is ONE
//    v_exp_f32 per score and no per-tile row max exists (fwd_tile).
//  * K/V tiles of 64 keys staged through LDS (double buffer, register staging: tile t+1's global
//    loads are in flight during tile t's MFMAs), one barrier per tile.
//  * S^T = K Q^T with v_mfma_f32_32x32x16_bf16 (query on the lane: the row sums are lane-local;
//    the two 32-key halves meet once, after the last tile); P converted to bf16 in registers is
//    the B operand of O^T = V^T P^T, V^T read with ds_read_b64_tr_b16 in the matching key order.
//  * dropout: lane masks from attn_dropmask_kernel (scalar loads, one v_cndmask per score).
template <int NKS, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const AttnArgs a) {
  constexpr int NH = (NKS + 3) / 4;   // 64-column halves of the LDS images
  constexpr int NO = (NKS + 1) / 2;   // 32-column O^T accumulator tiles
  constexpr int HALF = 64 * ROWB;     // one 64-row, 64-column image
  constexpr int TILE = NH * HALF;     // one K or V tile
  constexpr int NC = 2 * NH;          // 16-byte chunks per thread per tile per matrix
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 V0 K1 V1
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h32 = lane >> 5, l32 = lane & 31;
  const int nqb = (a.T + 127) / 128;
  const int npair = (nqb + 1) / 2;
  const int BH = a.B * a.H;
  int bh, pr;
  if (!MG_FWD_PAIR) {  // one query block per workgroup, heaviest blocks first
    bh = blockIdx.x % BH;
    pr = blockIdx.x / BH;
  } else if ((BH & 7) == 0) {  // (b, h)'s workgroups 8 apart: one XCD
    const int x = blockIdx.x & 7, rest = blockIdx.x >> 3;
    pr = rest % npair;
    bh = (rest / npair) * 8 + x;
  } else {
    pr = blockIdx.x % npair;
    bh = blockIdx.x / npair;
  }
  const int b = bh / a.H, hh = bh % a.H;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  // the pair's query blocks, heavier first; the middle block of an odd count runs alone
  const int qbA = nqb - 1 - pr, qbB = pr;
  const bool two = MG_FWD_PAIR && qbB < qbA;
  const int ntA = (min(a.T, qbA * 128 + 128) + 63) / 64;
  const int ntB = two ? (min(a.T, qbB * 128 + 128) + 63) / 64 : 0;
  const int nt = (a.T + 63) / 64;

  // tile staging: chunk c of this thread -> (half, row, 16-byte column chunk), offsets once.  The
  // loads are buffer loads through a per-tile descriptor (base = the tile's first key row, extent
  // = the rest of qkv): no per-lane bounds branches or 64-bit address math per tile.  Rows past T
  // read the next sequence's (finite) rows or, past the tensor, zeros; their scores are masked
  // (the tile takes the masked body) and their p is 0.  Columns past hd read the neighbouring
  // head: K there meets zero Q columns, V there only feeds O columns that are never stored.
  uint32_t voff[NC], sdst[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + 256 * c;
    const int hf = idx >> 9, rem = idx & 511;
    voff[c] = (uint32_t)(((rem >> 3) * ld + hf * 64 + (rem & 7) * 8) * 2);
    sdst[c] = hf * HALF + lds_off(rem >> 3, rem & 7);
  }
  const uint64_t kv_bytes = (uint64_t)a.B * a.T * ld * 2;  // the whole qkv tensor
  const uint64_t kbase = (uint64_t)((const char*)Kg - (const char*)a.qkv);
  auto load_tile = [&](uint4 (&rk)[NC], uint4 (&rv)[NC], int k0) {
    const uint64_t off = kbase + (uint64_t)k0 * ld * 2;
    const __amdgpu_buffer_rsrc_t dk = kv_rsrc(a.qkv, kv_bytes, off);
    const __amdgpu_buffer_rsrc_t dv = kv_rsrc(a.qkv, kv_bytes, off + (uint64_t)a.D * 2);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      rk[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dk, voff[c], 0, 0));
      rv[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dv, voff[c], 0, 0));
    }
  };
  auto store_tile = [&](char* dst, const uint4 (&rk)[NC], const uint4 (&rv)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      *reinterpret_cast<uint4*>(dst + sdst[c]) = rk[c];
      *reinterpret_cast<uint4*>(dst + TILE + sdst[c]) = rv[c];
    }
  };

  // per-lane fragment offsets: K rows l32 (+32 per sub: an immediate), chunk 2 ks + h32;
  // V^T transposed reads rows 4 h32 + q (+8), columns (n & 1) * 32 + cb + 4 p
  int ko[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) ko[ks] = (ks >> 2) * HALF + lds_off(l32, (2 * ks + h32) & 7);
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int ta0 = tr_off(4 * h32 + trq, trc), tb0 = tr_off(8 + 4 * h32 + trq, trc);
  const int ta1 = tr_off(4 * h32 + trq, 32 + trc), tb1 = tr_off(8 + 4 * h32 + trq, 32 + trc);

  bf16x8 qf[NKS];
  f32x16 o[NO], negm;
  float m = 0.f, l = 0.f;
  int q0 = 0, myq = 0;
  auto begin_block = [&](int qb) {  // Q fragments (k-step ks: columns 16 ks + 8 h32 .. +7), scaled
    q0 = qb * 128;
    myq = q0 + 32 * w + l32;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d = ks * 16 + 8 * h32;
      uint4 u = (myq < a.T && d < a.hd) ? ld16(Qg + (long)myq * ld + d) : make_uint4(0, 0, 0, 0);
      float f[8];
      unpack8(u, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= a.scale_log2;
      qf[ks] = __builtin_bit_cast(bf16x8, pack8(f));
    }
#pragma unroll
    for (int n = 0; n < NO; ++n) o[n] = f32x16{0};
    negm = f32x16{0};
    m = 0.f;
    l = 0.f;
  };
  auto end_block = [&]() {
    const float lt = sum_xor32(l);
    if (myq < a.T) {
      const float inv = (DROP ? a.dscale : 1.f) / lt;
      if (h32 == 0) a.lse[(long)bh * a.T + myq] = m + log2f(lt);  // log2 domain
      bf16_t* orow = a.out + ((long)b * a.T + myq) * a.D + hh * a.hd;
#pragma unroll
      for (int n = 0; n < NO; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = n * 32 + 8 * g + 4 * h32;
          if (d < a.hd)
            *reinterpret_cast<uint2*>(orow + d) = make_uint2(pack2(o[n][4 * g] * inv, o[n][4 * g + 1] * inv),
                                                             pack2(o[n][4 * g + 2] * inv, o[n][4 * g + 3] * inv));
        }
    }
  };

  // row-word dropout: word (bh, 2 t + h32, q) of this lane's query, loaded one tile ahead
  auto row_word = [&](int t, int q) -> uint32_t {
    return a.dmask[((long)bh * (2 * nt) + 2 * t + h32) * a.T + min(q, a.T - 1)];
  };
  begin_block(qbA);
  uint32_t kw_next = DROP ? row_word(0, myq) : 0u;
  {
    uint4 rk[NC], rv[NC];
    load_tile(rk, rv, 0);
    store_tile(smem, rk, rv);
  }
  __syncthreads();
  const int nall = ntA + ntB;
  for (int it = 0; it < nall; ++it) {
    const bool second = it >= ntA;
    const int t = second ? it - ntA : it;
    const char* sk = smem + (it & 1) * 2 * TILE;
    const char* sv = sk + TILE;
    const bool more = it + 1 < nall;
    uint4 rk[NC], rv[NC];
    if (more) load_tile(rk, rv, (it + 1 == ntA ? 0 : t + 1) * 64);
    uint32_t kw_cur = kw_next;
    if (DROP && more) {  // next tile's keep words, a tile ahead (latency hidden)
      const bool seam = it + 1 == ntA;
      kw_next = row_word(seam ? 0 : t + 1, seam ? qbB * 128 + 32 * w + l32 : myq);
    }
    const int k0 = t * 64;
    const int wave_q = q0 + 32 * w;
    if (k0 <= wave_q + 31 && wave_q < a.T) {  // (a wave past the sequence end has nothing to do)
      const int lim = min(myq, a.T - 1) - k0 - 4 * h32;
      // causal / sequence-end mask only on the tiles that need it (separate bodies: a uniform
      // branch inside one body got if-converted into compares + selects on every tile)
      const bool diag = k0 + 63 > wave_q || k0 + 64 > a.T;
      if (diag) fwd_tile<NKS, true, DROP>(sk, sv, ko, qf, o, negm, m, l, t == 0, kw_cur, lim, ta0, tb0, ta1, tb1);
      else fwd_tile<NKS, false, DROP>(sk, sv, ko, qf, o, negm, m, l, t == 0, kw_cur, lim, ta0, tb0, ta1, tb1);
    }
    if (it + 1 == ntA) {  // seam: first block done, the second starts with the prefetched tile 0
      end_block();
      if (two) begin_block(qbB);
    }
    if (more) store_tile(smem + ((it + 1) & 1) * 2 * TILE, rk, rv);
    __syncthreads();
  }
  if (two) end_block();
}

// max of three floats in one v_max3_f32 (inline asm: hipcc canonicalises MFMA results with an
// extra v_max_f32 x, x before each fmaxf)
MG_DEVICE float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// keep mask of packed pair j (bf16x2 word j of a lane's P operand): bits j and 16 + j of the
// row word, each sign-extended over its 16-bit half (one shift + one v_pk_ashrrev_i16)
MG_DEVICE uint32_t pair_mask(uint32_t kw, int j) {
  const s16x2 mk = __builtin_bit_cast(s16x2, kw << (15 - j)) >> (s16x2){15, 15};
  return __builtin_bit_cast(uint32_t, mk);
}

// =============================================================================== pipelined forward
// Forward for head dims up to 64 (NKS <= 4: one 64-column LDS image), software-pipelined inside
// each wave so that one tile's softmax VALU issues while the NEXT tile's QK^T MFMAs are in flight:
//
//   iteration t:  S(t+1) = (cK(t+1)) Q^T - m   [8 MFMAs, issued first]
//                 softmax(t): range check (max3), exp2, pack P (bf16 pairs), dropout mask on the
//                 packed pairs                    [VALU, overlaps the MFMAs above]
//                 O^T += V^T (Z P)^T, l^T += 1^T P^T [MFMAs; the row sum runs on the matrix pipe]
//                 stage K(t+2), V(t+1) (register staging), one barrier
//
//  * workgroup = 4 waves = 128 queries of one (b, h); 2 workgroups per CU (two waves per SIMD,
//    from different workgroups, so one wave's softmax and the other's MFMAs interleave too).
//  * the running max m rides in as the S MFMA's C operand, so p = exp2(S') is one v_exp_f32; m
//    moves only when a tile's scores leave [-64, 64] (log2 units) -- rare after the first tile of
//    a block; then o, l and the already-issued next tile are rescaled in place (no recompute).
//  * the row sum l = sum of the undropped bf16 P is an MFMA against a ones operand (4 per tile)
//    instead of 32 VALU adds per lane: the matrix pipe has the slack, the vector pipe does not.
//  * dropout on the packed bf16 P: pair j's keep bits sit at j and 16 + j of the lane's row
//    word (drop_bit), so its 32-bit mask is one shift + one v_pk_ashrrev_i16 and the drop one AND
//    per pair (1.5 VALU per score; was a bit-field extract + AND per fp32 score).
//  * the causal mask touches only each wave's last (diagonal) tile.
//  * the workgroups of one (b, h) run 8 apart in the grid (one XCD under round-robin placement:
//    K / V shared through that XCD's L2), heaviest query block first within the group.
// (The round-4 timing-only ablations of this kernel -- outputs wrong on purpose -- live outside the
// production source: bench/dev/attn_ablations.patch, applied to a scratch copy by scripts/build_variant.sh.)
template <int NKS, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_pipe_kernel(const AttnArgs a) {
  static_assert(NKS >= 1 && NKS <= 4, "pipelined forward: head dim <= 64");
  constexpr int NO = (NKS + 1) / 2;  // 32-column O^T accumulator tiles
  constexpr int TILE = 64 * ROWB;    // one K or V tile (64 keys x 64 columns)
  constexpr int LM = NKS >= 3;       // row sum on the MFMA pipe (hd 33..64); VALU adds below
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 K1 V0 V1
  char* const sK = smem;
  char* const sV = smem + 2 * TILE;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h32 = lane >> 5, l32 = lane & 31;
  const int nqb = (a.T + 127) / 128;
  const int npair = (nqb + 1) / 2;
  const int BH = a.B * a.H;
  int bh, pr;
  if ((BH & 7) == 0) {  // the (b, h)'s workgroups 8 apart: one XCD (K / V shared in its L2)
    const int x = blockIdx.x & 7, rest = blockIdx.x >> 3;
    pr = rest % npair;
    bh = (rest / npair) * 8 + x;
  } else {
    pr = blockIdx.x % npair;
    bh = blockIdx.x / npair;
  }
  // two query blocks per workgroup, the pr-th heaviest then the pr-th lightest (every workgroup
  // the same causal work); the K / V tile stream runs on across the seam
  const int qbA = nqb - 1 - pr, qbB = pr;
  const int nblk = qbB < qbA ? 2 : 1;
  const int b = bh / a.H, hh = bh % a.H;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  const int ntA = (min(a.T, qbA * 128 + 128) + 63) / 64;
  const int ntB = nblk == 2 ? (min(a.T, qbB * 128 + 128) + 63) / 64 : 0;
  const int nall = ntA + ntB;  // unified tile stream: A's tiles, then B's

  // ---- K / V staging: thread chunk c -> (row, 16-byte column chunk); per-tile buffer descriptor
  uint32_t voff[2], sdst[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = threadIdx.x + 256 * c;
    voff[c] = (uint32_t)(((idx >> 3) * ld + (idx & 7) * 8) * 2);
    sdst[c] = lds_off(idx >> 3, idx & 7);
  }
  const uint64_t kv_bytes = (uint64_t)a.B * a.T * ld * 2;
  const uint64_t kbase = (uint64_t)((const char*)Kg - (const char*)a.qkv);
  // unified stream index u -> the (b, h)'s key tile
  auto src_tile = [&](int u) __attribute__((always_inline)) { return u < ntA ? u : u - ntA; };
  auto load_k = [&](uint4 (&r)[2], int u) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t d = kv_rsrc(a.qkv, kv_bytes, kbase + (uint64_t)src_tile(u) * 64 * ld * 2);
#pragma unroll
    for (int c = 0; c < 2; ++c) r[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(d, voff[c], 0, 0));
  };
  auto load_v = [&](uint4 (&r)[2], int u) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t d =
        kv_rsrc(a.qkv, kv_bytes, kbase + (uint64_t)src_tile(u) * 64 * ld * 2 + (uint64_t)a.D * 2);
#pragma unroll
    for (int c = 0; c < 2; ++c) r[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(d, voff[c], 0, 0));
  };
  auto store_tile = [&](char* dst, const uint4 (&r)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 2; ++c) *reinterpret_cast<uint4*>(dst + sdst[c]) = r[c];
  };

  // ---- per-lane fragment offsets: K rows l32 (+32 per sub), chunk 2 ks + h32; V^T transposed
  int ko[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) ko[ks] = lds_off(l32, 2 * ks + h32);
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int ta0 = tr_off(4 * h32 + trq, trc), tb0 = tr_off(8 + 4 * h32 + trq, trc);
  const int ta1 = tr_off(4 * h32 + trq, 32 + trc), tb1 = tr_off(8 + 4 * h32 + trq, 32 + trc);
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));

  // ---- prologue staging: K(0), V(0), K(1) loads in flight together, then K(2), V(1) into the
  // staging registers (written at iteration 0's start)
  uint4 rk[2], rv[2];
  {
    uint4 rk1[2];
    load_k(rk, 0);
    load_v(rv, 0);
    load_k(rk1, min(1, nall - 1));
    store_tile(sK, rk);
    store_tile(sV, rv);
    store_tile(sK + TILE, rk1);
  }
  load_k(rk, min(2, nall - 1));
  load_v(rv, min(1, nall - 1));
  __syncthreads();

  for (int bi = 0; bi < nblk; ++bi) {
    const int qb = bi ? qbB : qbA;
    const int u0 = bi ? ntA : 0;  // stream index of the block's tile 0
    const int q0 = qb * 128;
    const int qw = q0 + 32 * w;                                 // this wave's first query
    const int myq = qw + l32;
    const int tw = qw < a.T ? min(a.T - 1, qw + 31) / 64 : -1;  // this wave's last (diagonal) tile

    // Q fragments (k-step ks: columns 16 ks + 8 h32 .. +7), pre-scaled into the log2 domain
    bf16x8 qf[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d = ks * 16 + 8 * h32;
      uint4 u = (myq < a.T && d < a.hd) ? ld16(Qg + (long)myq * ld + d) : make_uint4(0, 0, 0, 0);
      float f[8];
      unpack8(u, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= a.scale_log2;
      qf[ks] = __builtin_bit_cast(bf16x8, pack8(f));
    }
    f32x16 o[NO], lacc = f32x16{0}, negm = f32x16{0};
#pragma unroll
    for (int n = 0; n < NO; ++n) o[n] = f32x16{0};
    float m = 0.f, lv = 0.f;

    // keep word of tile t (this lane's 32 scores), clamped query row for padding lanes
    auto row_word = [&](int t) -> uint32_t __attribute__((always_inline)) {
      return a.dmask[((long)bh * (2 * ((a.T + 63) / 64)) + 2 * t + h32) * a.T + min(myq, a.T - 1)];
    };
    // S(t) = (cK(t)) Q^T - m for the wave's 32 queries x the tile's 64 keys (key on the row);
    // the accumulators are separate named vectors (arrays of them passed around went to scratch)
    auto scores = [&](f32x16& s0, f32x16& s1, const char* sk) __attribute__((always_inline)) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk, ko[0]), qf[0], negm, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk + 32 * ROWB, ko[0]), qf[0], negm, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < NKS; ++ks) {
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk, ko[ks]), qf[ks], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sk + 32 * ROWB, ko[ks]), qf[ks], s1, 0, 0, 0);
      }
    };
    // causal mask of a wave's diagonal tile t: key 64 t + k0 + 4 h32 + (r & 3) + 8 (r >> 2) > query
    // -> -inf (p = 0).  Applied to S(t) once, right after its MFMAs were issued.
    auto mask_diag = [&](f32x16& c0, f32x16& c1, int t) __attribute__((always_inline)) {
      const int lim = myq - 64 * t - 4 * h32;
      auto mask = [&](f32x16& c, int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) c[r] = (k0 + (r & 3) + 8 * (r >> 2) > lim) ? -__builtin_huge_valf() : c[r];
      };
      mask(c0, 0);
      mask(c1, 32);
    };
    // p = exp2(S') packed to bf16 pairs (the P^T operand layout of the PV MFMA); rs += sum (hd <= 32)
    auto expack = [&](const f32x16& c, int st, float& rs) __attribute__((always_inline)) -> bf16x8 {
      uint32_t u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p0 = fexp2(c[8 * st + 2 * i]), p1 = fexp2(c[8 * st + 2 * i + 1]);
        if (!LM) rs += p0 + p1;
        u[i] = pack2(p0, p1);
      }
      return __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    };
    // dropped P: pair j's mask = sign-extended bits j / 16 + j of the row word
    auto dropped = [&](const bf16x8& pu, int j, uint32_t kw) __attribute__((always_inline)) -> bf16x8 {
      if constexpr (!DROP) return pu;
      const uint4 u = __builtin_bit_cast(uint4, pu);
      return __builtin_bit_cast(bf16x8, make_uint4(u.x & pair_mask(kw, j), u.y & pair_mask(kw, j + 1),
                                                   u.z & pair_mask(kw, j + 2), u.w & pair_mask(kw, j + 3)));
    };

    // One tile of one wave: S(t+1) issued first (speculative on the diagonal tile), then S(t)'s
    // range check, exp2, packing and dropout (VALU beside those MFMAs), the rare rescale, then
    // O^T += V^T (Z P)^T and l^T += 1^T P^T.
    // DIAG: the wave's last (diagonal) tile t == tw: S(t) masked in place first, no S(t+1)
    auto compute = [&](f32x16& c0, f32x16& c1, f32x16& n0, f32x16& n1, int t, uint32_t kw, auto diag_tag) __attribute__((always_inline)) {
      constexpr bool DIAG = decltype(diag_tag)::value;
      const int u = u0 + t;
      const char* sv = sV + (u & 1) * TILE;
      if constexpr (DIAG) mask_diag(c0, c1, t);
      else scores(n0, n1, sK + ((u + 1) & 1) * TILE);
      float mx = max3f(c0[0], c0[1], c0[2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) mx = max3f(mx, c0[r], c0[r + 1]);
      mx = max3f(mx, c0[15], c1[0]);
#pragma unroll
      for (int r = 1; r < 15; r += 2) mx = max3f(mx, c1[r], c1[r + 1]);
      mx = fmaxf(mx, c1[15]);
      float rs = 0.f;
      bf16x8 pu00 = expack(c0, 0, rs), pu01 = expack(c0, 1, rs), pu10 = expack(c1, 0, rs), pu11 = expack(c1, 1, rs);
      // pinned before the range-check branch, so the exp2 / pack VALU stays beside the S(t+1)
      // MFMAs (hipcc otherwise sinks it below the branch into the PV block)
      asm volatile("" ::"v"(pu00), "v"(pu01), "v"(pu10), "v"(pu11));
      const bool first = t == 0;
      if (__builtin_expect(__any(mx > 64.f || (first && mx < -64.f)), 0)) {
        // row max over both halves; a block's first tile may move m down (nothing accumulated yet)
        const float mr = max_xor32(mx);
        const float d = first ? mr : fmaxf(mr, 0.f);
        const float alpha = fexp2(-d);
#pragma unroll
        for (int n = 0; n < NO; ++n) o[n] *= alpha;
        lacc *= alpha;
        lv *= alpha;
        m += d;
        negm = -m;
        c0 -= d;
        c1 -= d;
        if constexpr (!DIAG) {
          n0 -= d;  // S(t+1) was issued against the old m
          n1 -= d;
        }
        rs = 0.f;
        pu00 = expack(c0, 0, rs), pu01 = expack(c0, 1, rs), pu10 = expack(c1, 0, rs), pu11 = expack(c1, 1, rs);
      }
      if (!LM) lv += rs;
      const bf16x8 pd00 = dropped(pu00, 0, kw), pd01 = dropped(pu01, 4, kw), pd10 = dropped(pu10, 8, kw),
                   pd11 = dropped(pu11, 12, kw);
      auto pv = [&](const bf16x8& pd, const bf16x8& pu, int rb) __attribute__((always_inline)) {
#pragma unroll
        for (int n = 0; n < NO; ++n)
          o[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              (n & 1) ? lds_tr_at(sv + rb, ta1, tb1) : lds_tr_at(sv + rb, ta0, tb0), pd, o[n], 0, 0, 0);
        if (LM) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pu, lacc, 0, 0, 0);
      };
      pv(pd00, pu00, 0);  // 16-row aligned LDS row bases: immediates
      pv(pd01, pu01, 16 * ROWB);
      pv(pd10, pu10, 32 * ROWB);
      pv(pd11, pu11, 48 * ROWB);
    };

    // block prologue: S(0) from K(u0) (staged), then a barrier before anyone restages that slot
    uint32_t kw_cur = DROP ? row_word(0) : 0u;
    f32x16 sA0, sA1, sB0, sB1;
    if (tw >= 0) scores(sA0, sA1, sK + (u0 & 1) * TILE);
    __syncthreads();

    // iteration t (stream u = u0 + t): first write the staging registers -- K(u+2), V(u+1),
    // loaded one iteration ago -- into the slots K(u) / V(u-1) held (read before the previous
    // barrier) and re-issue them at once for K(u+3), V(u+2), so a load has a whole iteration and
    // its barrier to land; then softmax / PV of tile t from c (and S(t+1) -> n unless it is the
    // wave's diagonal tile).  Every load and store is unconditional (indices clamped; a stream
    // tile past the end lands in a slot nobody reads again): conditional loads made hipcc wait
    // vmcnt(0) ahead of the next iteration's loads -- a full memory latency per tile.
    const int nt = bi ? ntB : ntA;
    auto stage = [&](int t, auto&& body) __attribute__((always_inline)) {
      const int u = u0 + t;
      store_tile(sK + (u & 1) * TILE, rk);
      store_tile(sV + ((u + 1) & 1) * TILE, rv);
      load_k(rk, min(u + 3, nall - 1));
      load_v(rv, min(u + 2, nall - 1));
      const uint32_t kw_next = DROP ? row_word(min(t + 1, max(tw, 0))) : 0u;
      body();
      kw_cur = kw_next;
      __syncthreads();
    };
    // Per wave: steady tiles t < tw, the diagonal tile tw, then idle tiles up to the workgroup's
    // nt.  The trip counts differ between waves but every iteration has exactly one barrier, so
    // waves 0-1 at their diagonal meet waves 2-3 at their last steady tile.  No iteration body
    // holds both compute variants (a steady / diagonal branch inside one body spilled).
    int t = 0;
    if (tw >= 0) {
      for (; t + 1 < tw; t += 2) {
        stage(t, [&]() __attribute__((always_inline)) { compute(sA0, sA1, sB0, sB1, t, kw_cur, std::false_type{}); });
        stage(t + 1, [&]() __attribute__((always_inline)) { compute(sB0, sB1, sA0, sA1, t + 1, kw_cur, std::false_type{}); });
      }
      if (t < tw) {  // odd count: one more steady tile; S(tw) then sits in the B set
        stage(t, [&]() __attribute__((always_inline)) { compute(sA0, sA1, sB0, sB1, t, kw_cur, std::false_type{}); });
        ++t;
        sA0 = sB0;
        sA1 = sB1;
      }
      stage(t, [&]() __attribute__((always_inline)) { compute(sA0, sA1, sB0, sB1, t, kw_cur, std::true_type{}); });
      ++t;
    }
    for (; t < nt; ++t) stage(t, []() {});

    // block epilogue: O = o * dscale / l, lse = m + log2 l (log2 domain)
    if (myq < a.T) {
      const float lt = LM ? lacc[0] : sum_xor32(lv);
      const float inv = (DROP ? a.dscale : 1.f) / lt;
      if (h32 == 0) a.lse[(long)bh * a.T + myq] = m + log2f(lt);
      bf16_t* orow = a.out + ((long)b * a.T + myq) * a.D + hh * a.hd;
#pragma unroll
      for (int n = 0; n < NO; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = n * 32 + 8 * g + 4 * h32;
          if (d < a.hd)
            *reinterpret_cast<uint2*>(orow + d) = make_uint2(pack2(o[n][4 * g] * inv, o[n][4 * g + 1] * inv),
                                                             pack2(o[n][4 * g + 2] * inv, o[n][4 * g + 3] * inv));
        }
    }
  }
}

}  // namespace

namespace mg {

// row words [B*H][2 ceil(T/64)][T] u32 (attn_dropmask_kernel)
size_t attention_dropout_mask_words(int B, int T, int H) { return (size_t)B * H * T * 2 * ((T + 63) / 64); }

int attention_dropout_threshold(float p) {
  // 16-bit dropout threshold: effective p = thr / 65536 (0.1 -> 0.100006)
  if (!(p > 0.f)) return 0;
  const long thr = lrint((double)p * 65536.0);
  return (int)(thr < 1 ? 1 : (thr > 65535 ? 65535 : thr));
}

float attention_dropout_scale(int thr) { return thr ? 65536.f / (65536.f - (float)thr) : 1.f; }

void attention_dropout_mask(uint32_t* dmask, int B, int T, int H, float p, uint64_t seed,
                            hipStream_t stream) {
  const int thr = attention_dropout_threshold(p);
  if (!thr) return;
  const int ntw = 2 * ((T + 63) / 64), ng = (T + 31) / 32, nt = (T + 63) / 64;
  attn_dropmask_kernel<<<dim3((unsigned)(B * H), (unsigned)cdiv(ng, 4)), 256, 0, stream>>>(
      dmask, B * H, T, ntw, ng, nt, seed, graph_seed_ofs(), (uint32_t)thr);
}

template <int NKS>
static void launch_fwd(const AttnArgs& a, int grid, hipStream_t stream) {
  if (a.thr) attn_fwd_kernel<NKS, true><<<grid, 256, 0, stream>>>(a);
  else attn_fwd_kernel<NKS, false><<<grid, 256, 0, stream>>>(a);
}

// MINGPT_ATTN_FWD_PIPE=0 keeps the round-3 kernel for hd <= 64 too (A/B only)
static bool use_pipe() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MINGPT_ATTN_FWD_PIPE");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

template <int NKS>
static void launch_fwd_pipe(const AttnArgs& a, hipStream_t stream) {
  const int grid = (cdiv(a.T, 128) + 1) / 2 * a.B * a.H;  // pairs of query blocks
  if (a.thr) attn_fwd_pipe_kernel<NKS, true><<<grid, 256, 0, stream>>>(a);
  else attn_fwd_pipe_kernel<NKS, false><<<grid, 256, 0, stream>>>(a);
}

void attention_fwd(const bf16_t* qkv, bf16_t* out, float* lse, uint32_t* dmask, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream) {
  AttnArgs a{};
  a.B = B; a.T = T; a.H = H; a.hd = hd; a.D = H * hd;
  a.scale_log2 = 1.4426950408889634f / sqrtf((float)hd);
  a.thr = dmask ? (uint32_t)attention_dropout_threshold(p) : 0u;
  a.dscale = attention_dropout_scale((int)a.thr);
  a.qkv = qkv; a.out = out; a.lse = lse; a.dmask = dmask;
  if (a.thr) attention_dropout_mask(dmask, B, T, H, p, seed, stream);
  const int nqb = cdiv(T, 128);
  const int grid = (MG_FWD_PAIR ? (nqb + 1) / 2 : nqb) * B * H;  // (pairs of) query blocks
  if (use_pipe() && nks_for(hd) <= 4) {
    switch (nks_for(hd)) {
      case 1: launch_fwd_pipe<1>(a, stream); return;
      case 2: launch_fwd_pipe<2>(a, stream); return;
      case 3: launch_fwd_pipe<3>(a, stream); return;
      default: launch_fwd_pipe<4>(a, stream); return;
    }
  }
  switch (nks_for(hd)) {
    case 1: launch_fwd<1>(a, grid, stream); break;
    case 2: launch_fwd<2>(a, grid, stream); break;
    case 3: launch_fwd<3>(a, grid, stream); break;
    case 4: launch_fwd<4>(a, grid, stream); break;
    case 6: launch_fwd<6>(a, grid, stream); break;
    default: launch_fwd<8>(a, grid, stream); break;
  }
}

}  // namespace mg
