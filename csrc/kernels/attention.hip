// Causal flash attention, forward and backward, for gfx950 (CDNA4, MI355X).
//
// Replaces the reference's nn.MultiheadAttention math path
// (/root/reference/mingpt/model.py:147-165: in-proj split, q*scale, baddbmm with the [T,T] mask,
// softmax, dropout, bmm PV, plus the discarded head-averaged weights) with a true causal kernel
// that never materialises [T, T] (fixes D4: the reference's additive 0/1 mask was not causal).
//
// I/O layout: qkv [B*T, 3*D] bf16 straight from the c_attn GEMM (q | k | v, head h at columns
// h*hd..), out [B*T, D] bf16, lse [B*H*T] fp32 (log2 domain).  hd <= 64 (every GPT-2 size is 64;
// gpt-mini/micro are 32, gpt-nano 16): tiles are 64 wide and zero-padded.
//
// Forward (FA2 structure, MI355X mapping):
//  * workgroup = 4 waves = 128 queries of one (b, h); each wave owns 32 queries.
//  * Q fragments live in VGPRs for the whole kernel; K/V tiles of 64 keys are staged through LDS
//    (double buffer, loads for tile t+1 issued before the MFMAs of tile t).
//  * S^T = K Q^T with v_mfma_f32_32x32x16_bf16 ("swapped" operands): the query is on the lane,
//    so the softmax row statistics are lane-local (one xor-32 shuffle joins the two halves).
//  * P is converted to bf16 in registers and used directly as the B operand of O^T = V^T P^T
//    (guide §3 "accumulator tile as the next MFMA's operand"); V^T fragments come from LDS with
//    ds_read_b64_tr_b16 in the matching permuted key order.  O^T keeps queries on the lane too,
//    so the online-softmax rescale is a per-lane multiply.
//  * LDS images use a 128-B-row XOR swizzle that is bank-conflict-free for both the row reads
//    (ds_read_b128) and the transposed reads (found by exhaustive search, see PERF.md).
//  * heaviest (last) query blocks are launched first; fully-masked K tiles are skipped per wave.
//
// Backward (key-block parallel):
//  * workgroup = 4 waves = 128 keys of one (b, h); each wave keeps its 32 keys' K and V fragments
//    in VGPRs and dK^T/dV^T accumulators (keys on the lane) across the whole query sweep.
//  * per 64-query tile (Q, dO, lse, delta staged in LDS): S and dP with the key on the lane, P and
//    dS in registers feed dV^T += dO^T P and dK^T += Q^T dS directly (tr-reads of Q/dO);
//    dS is transposed once through LDS for dQ = dS K, the 4 waves' dQ partials are summed with
//    LDS float atomics, then one fp32 global atomic per element per workgroup.
//  * attention dropout: Philox mask regenerated from (seed, b, h, q, key) in both passes.
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int HD = 64;        // tile head dim
constexpr int ROWB = HD * 2;  // 128-B LDS rows
constexpr float kNegBig = -1e30f;

// conflict-free for ds_read_b128 (32-row operand) and both ds_read_b64_tr_b16 patterns
MG_DEVICE int swz(int r) { return ((r >> 1) & 3) | ((((r >> 1) ^ (r >> 3)) & 1) << 2); }
MG_DEVICE int lds_off(int row, int ch) { return row * ROWB + ((ch ^ swz(row)) << 4); }

struct AttnArgs {
  const bf16_t* qkv;
  bf16_t* out;
  float* lse;          // [B*H*T], log2 domain
  const bf16_t* dout;  // bwd
  const float* delta;  // bwd [B*H*T]
  float* dq;           // bwd fp32 dQ: [B*T, D] atomic accumulator, or per-key-block partials
  long dq_part;        // bwd256: elements between key-block partials of dq (plain stores)
  bf16_t* dqkv;        // bwd [B*T, 3D]
  uint32_t* dmask;     // dropout keep-bits [B*H*T][2*ceil(T/64)] (fwd writes, bwd reads)
  int B, T, H, hd, D;
  float scale_log2;    // log2(e) / sqrt(hd)
  uint64_t seed;
  uint32_t seed_key;   // fwd dropout hash key derived from seed
  const uint64_t* sofs;  // hipGraph mode: seed_key is derived on the device (common.h eff_seed)
  uint32_t thr;        // 8-bit keep threshold: keep iff random byte >= thr (0 = no dropout)
  float dscale;        // 1 / (1 - thr/256)
  uint32_t kadd;       // SWAR keep test: 4 x (128 - thr) if thr <= 128, else 4 x (256 - thr)
};

MG_DEVICE float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }  // v_exp_f32, no denorm fixup

// 32-bit avalanche mixer (xorshift-multiply, "lowbias32" constants): a bijection with good
// avalanche, 5 VALU ops; the attention-dropout bytes are mix32 of distinct counters.
MG_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

MG_DEVICE bf16x8 lds_row_frag(const char* base, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(base + lds_off(row, ch));
}

// Transposed 8-element fragment: column col of rows r0..r0+3 (elements 0..3) and r1..r1+3 (4..7).
// Lane (in its 16-lane group) 4q+p addresses row r?+q, columns colbase+4p..+3.
MG_DEVICE bf16x8 lds_tr_frag(const char* base, int r0, int r1, int colbase, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = colbase + 4 * p;
  const int ra = r0 + q, rb = r1 + q;
  const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(base + lds_off(ra, col >> 3) + (col & 7) * 2));
  const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(base + lds_off(rb, col >> 3) + (col & 7) * 2));
  const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Byte offset of a transposed-read lane address (row, column) in an lds_off image.
MG_DEVICE int tr_off(int row, int col) { return lds_off(row, col >> 3) + (col & 7) * 2; }

// Transposed fragment from two precomputed per-lane offsets (rows r0+q and r0+8+q, or +4): the
// swizzle is periodic in the row with period 16, so a 16-row-aligned row base is a plain byte
// offset the caller passes as a compile-time constant (it lands in the ds_read offset field)
// instead of a per-read swizzle computation.
MG_DEVICE bf16x8 lds_tr_at(const char* base, int oa, int ob) {
  const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + oa));
  const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + ob));
  const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  return __builtin_bit_cast(bf16x8, v);
}

MG_DEVICE bf16x8 lds_row_at(const char* base, int o) { return *reinterpret_cast<const bf16x8*>(base + o); }

MG_DEVICE bf16x8 pack_frag(const f32x16& a, int s) {
  s16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(a[8 * s + j]);
  return __builtin_bit_cast(bf16x8, v);
}

// stage a [64 rows][64 cols] bf16 tile (rows r0.., column offset col0 in a row-major matrix with
// leading dimension ld) into registers: 512 chunks of 16 B, 2 per thread.
MG_DEVICE void load64(uint4 (&reg)[2], const bf16_t* base, long ld, int r0, int rows, int hd) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int row = idx >> 3, ch = idx & 7;
    const int r = r0 + row;
    reg[i] = (r < rows && ch * 8 < hd) ? ld16(base + (long)r * ld + ch * 8) : make_uint4(0, 0, 0, 0);
  }
}

MG_DEVICE void store64(char* lds, const uint4 (&reg)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    *reinterpret_cast<uint4*>(lds + lds_off(idx >> 3, idx & 7)) = reg[i];
  }
}

// =============================================================================== forward
template <int NKS>  // head-dim tile = 16 * NKS (hd zero-padded up to it)
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 64 * ROWB];  // K0 V0 K1 V1
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h32 = lane >> 5, l32 = lane & 31;
  const int nqb = (a.T + 127) / 128;
  const int bh = blockIdx.x % (a.B * a.H);
  const int qb = nqb - 1 - blockIdx.x / (a.B * a.H);  // heaviest blocks first
  const int b = bh / a.H, hh = bh % a.H;
  const int q0 = qb * 128;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  const bf16_t* Vg = Qg + 2 * a.D;

  const int myq = q0 + 32 * w + l32;
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int d = ks * 16 + 8 * h32;
    uint4 u = (myq < a.T && d < a.hd) ? ld16(Qg + (long)myq * ld + d) : make_uint4(0, 0, 0, 0);
    qf[ks] = __builtin_bit_cast(bf16x8, u);
  }
  f32x16 o0 = {0}, o1 = {0};
  float m = kNegBig, l = 0.f;
  const int kend = min(a.T, q0 + 128);
  const int ntiles = (kend + 63) / 64;
  const int wave_qmax = q0 + 32 * w + 31;
  const uint64_t drop_row = (uint64_t)bh * a.T + myq;
  const int ntiles_all = (a.T + 63) / 64;
  uint32_t seed_key = a.seed_key;
  if (a.sofs) {  // same derivation as make_args, from this replay's seed
    const uint64_t sd = eff_seed(a.seed, a.sofs);
    seed_key = mix32((uint32_t)sd) ^ mix32((uint32_t)(sd >> 32) + 0x9E3779B9u);
  }

  uint4 rk[2], rv[2];
  load64(rk, Kg, ld, 0, a.T, a.hd);
  load64(rv, Vg, ld, 0, a.T, a.hd);
  store64(smem, rk);
  store64(smem + 64 * ROWB, rv);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const char* sk = smem + (t & 1) * 2 * 64 * ROWB;
    const char* sv = sk + 64 * ROWB;
    const bool more = t + 1 < ntiles;
    if (more) {
      load64(rk, Kg, ld, (t + 1) * 64, a.T, a.hd);
      load64(rv, Vg, ld, (t + 1) * 64, a.T, a.hd);
    }
    const int k0 = t * 64;
    if (k0 <= wave_qmax) {
      f32x16 s[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        s[sub] = f32x16{0};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
          s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              lds_row_frag(sk, sub * 32 + l32, ks * 2 + h32), qf[ks], s[sub], 0, 0, 0);
      }
      // mask only the tiles that need it (diagonal / past T: wave-uniform), row max on raw scores
      const bool diag = k0 + 63 > q0 + 32 * w;
      if (diag || k0 + 64 > a.T) {
        // key = k0 + c(sub, r) + 4 h32 with c a constant: one compare against a per-lane limit
        const int lim = min(myq, a.T - 1) - k0 - 4 * h32;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            s[sub][r] = (sub * 32 + (r & 3) + 8 * (r >> 2) > lim) ? kNegBig : s[sub][r];
      }
      float mx = s[0][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[1][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // online softmax; the O / l rescale runs only when some lane's max grew (exact: lanes whose
      // max did not grow get alpha = 1), which after the first few tiles is rare
      if (__any(mx > m)) {
        const float mn = fmaxf(m, mx);
        const float alpha = fexp2((m - mn) * a.scale_log2);
        m = mn;
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
      }
      // p = exp2(s * c - m * c): the softmax scale folded into one FMA per element
      const float mc = m * a.scale_log2;
      float rs = 0.f;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(__builtin_fmaf(s[sub][r], a.scale_log2, -mc));
          s[sub][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      l += rs;
      if (a.thr) {  // attention dropout on P (for O only; l uses the undropped P)
        // 32 random bytes per lane and tile from a counter hash (the keep bits are stored for the
        // backward, so this generator never has to be replayed elsewhere); keep iff byte >= thr.
        // The keep scale 1/(1-p) is applied once to O at the end.
        const uint64_t ctr = (drop_row * (uint64_t)ntiles_all + t) * 2 + h32;
        const uint32_t base = mix32((uint32_t)ctr ^ mix32((uint32_t)(ctr >> 32) ^ seed_key));
        uint32_t rw[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) rw[i] = mix32(base + (uint32_t)i * 0x9E3779B9u);
        // SWAR keep test on 4 bytes at once: bit 7 of each byte <- (byte >= thr); the keep word
        // gets element e = 4i + j (byte j of rw[i]) at bit 8j + i
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t x = rw[i];
          const uint32_t y = (x & 0x7f7f7f7fu) + a.kadd;
          const uint32_t k7 = (a.thr <= 128 ? (y | x) : (y & x)) & 0x80808080u;
          bits |= k7 >> (7 - i);
        }
#pragma unroll
        for (int e = 0; e < 32; ++e) {
          const int keep = __builtin_amdgcn_sbfe((int)bits, 8 * (e & 3) + (e >> 2), 1);  // 0 / -1
          s[e >> 4][e & 15] = __int_as_float(__float_as_int(s[e >> 4][e & 15]) & keep);
        }
        if (myq < a.T) a.dmask[(long)drop_row * (2 * ntiles_all) + t * 2 + h32] = bits;
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pf = pack_frag(s[sub], st);
          const int r0 = sub * 32 + 16 * st + 4 * h32;
          const int cb = 16 * ((lane >> 4) & 1);
          o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sv, r0, r0 + 8, cb, lane), pf, o0, 0, 0, 0);
          if constexpr (NKS > 2)
            o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sv, r0, r0 + 8, 32 + cb, lane), pf, o1, 0, 0, 0);
        }
    }
    if (more) {
      char* dst = smem + ((t + 1) & 1) * 2 * 64 * ROWB;
      store64(dst, rk);
      store64(dst + 64 * ROWB, rv);
    }
    __syncthreads();
  }

  if (myq < a.T) {
    const float inv = (a.thr ? a.dscale : 1.f) / l;
    if (h32 == 0) a.lse[(long)bh * a.T + myq] = m * a.scale_log2 + log2f(l);  // log2 domain
    bf16_t* orow = a.out + ((long)b * a.T + myq) * a.D + hh * a.hd;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 8 * g + 4 * h32;
      if (d < a.hd)
        *reinterpret_cast<uint2*>(orow + d) =
            make_uint2(pack2(o0[4 * g] * inv, o0[4 * g + 1] * inv), pack2(o0[4 * g + 2] * inv, o0[4 * g + 3] * inv));
      if (32 + d < a.hd)
        *reinterpret_cast<uint2*>(orow + 32 + d) =
            make_uint2(pack2(o1[4 * g] * inv, o1[4 * g + 1] * inv), pack2(o1[4 * g + 2] * inv, o1[4 * g + 3] * inv));
    }
  }
}

// =============================================================================== backward
// delta[(b*H + h)*T + t] = sum_d dO * O.  One lane per 16-byte chunk (8 elements) of a head row,
// lanes of consecutive chunks/heads/tokens read contiguous memory; the hd/8 lanes of a head row
// are reduced with xor-shuffles (hd/8 is a power of two <= 8).
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ out,
                                                           float* __restrict__ delta, int B, int T,
                                                           int H, int hd, int D) {
  const int cpr = hd >> 3;  // chunks per head row: 1, 2, 4 or 8
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over B*T*D/8 chunks
  const long nchunks = (long)B * T * D / 8;
  float s = 0.f;
  if (i < nchunks) {
    float x[8], y[8];
    unpack8(ld16(dout + i * 8), x);
    unpack8(ld16(out + i * 8), y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
  for (int o = 1; o < cpr; o <<= 1) s += __shfl_xor(s, o, 64);
  if (i < nchunks && (i & (cpr - 1)) == 0) {
    const long e = i * 8;  // element index in [B*T, D]
    const long bt = e / D;
    const int hh = (int)((e % D) / hd);
    const int t = (int)(bt % T), b = (int)(bt / T);
    delta[((long)b * H + hh) * T + t] = s;
  }
}

constexpr int BQ = 64;  // queries per bwd tile
// LDS (single-buffered tiles; the next tile is prefetched in VGPRs while this one computes):
//   Q [64 q][64 d], dO [64 q][64 d], K block [128 keys][64 d], dS^T image [128 keys][64 q] (bf16),
//   lse/delta [2][64] f32, dropout keep-words [64 q][4] u32.
constexpr int BWD_Q_OFF = 0;
constexpr int BWD_DO_OFF = BWD_Q_OFF + BQ * ROWB;
constexpr int BWD_K_OFF = BWD_DO_OFF + BQ * ROWB;
constexpr int BWD_DS_OFF = BWD_K_OFF + 128 * ROWB;
constexpr int BWD_LD_OFF = BWD_DS_OFF + 128 * ROWB;
constexpr int BWD_MW_OFF = BWD_LD_OFF + 2 * BQ * 4;
constexpr int BWD_SMEM = BWD_MW_OFF + BQ * 4 * 4;  // 49.5 KiB

template <int NKS>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(const AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x >> 6;
  const int bh = blockIdx.x % (a.B * a.H);
  const int kb = blockIdx.x / (a.B * a.H);  // key block 0 (heaviest: sweeps all queries) first
  const int b = bh / a.H, hh = bh % a.H;
  const int kb0 = kb * 128;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  const bf16_t* Vg = Qg + 2 * a.D;
  const bf16_t* dOg = a.dout + (long)b * a.T * a.D + hh * a.hd;
  const float* lseg = a.lse + (long)bh * a.T;
  const float* dlg = a.delta + (long)bh * a.T;
  char* sK = smem + BWD_K_OFF;
  char* sdS = smem + BWD_DS_OFF;
  const float* sL = reinterpret_cast<const float*>(smem + BWD_LD_OFF);
  const uint32_t* sMW = reinterpret_cast<const uint32_t*>(smem + BWD_MW_OFF);

  int mykey, wave_kmin;
  bf16x8 vf[4];  // V^T fragments of this wave's keys stay in VGPRs; K fragments are re-read from sK
  {
    const int lane = threadIdx.x & 63, h32 = lane >> 5, l32 = lane & 31;
    mykey = kb0 + 32 * w + l32;
    wave_kmin = kb0 + 32 * w;
    uint4 r0[2], r1[2];
    load64(r0, Kg, ld, kb0, a.T, a.hd);
    load64(r1, Kg, ld, kb0 + 64, a.T, a.hd);
    store64(sK, r0);
    store64(sK + 64 * ROWB, r1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d = ks * 16 + 8 * h32;
      const bool ok = mykey < a.T && d < a.hd;
      vf[ks] = __builtin_bit_cast(bf16x8, ok ? ld16(Vg + (long)mykey * ld + d) : make_uint4(0, 0, 0, 0));
    }
  }
  // this lane's dropout bit inside the forward's keep-words (see attn_fwd_kernel)
  const int mw_col = (w >> 1) * 2 + ((mykey >> 2) & 1);
  const int mw_el = ((mykey & 32) >> 1) | (mykey & 3) | (((mykey >> 3) & 3) << 2);  // fwd element
  const int mw_bit = 8 * (mw_el & 3) + (mw_el >> 2);  // its bit in the keep word (attn_fwd_kernel)
  const int ntw = 2 * ((a.T + 63) / 64);
  const int t0w = (kb0 / 64) * 2;

  f32x16 dk0 = {0}, dk1 = {0}, dv0 = {0}, dv1 = {0};
  const int qt0 = kb0 / BQ;
  const int nqt = (a.T + BQ - 1) / BQ;

  uint4 rq[2], rd[2];
  float rl = 0.f;
  uint32_t rmw = 0;
  auto issue = [&](int qt) {
    load64(rq, Qg, ld, qt * BQ, a.T, a.hd);
    load64(rd, dOg, a.D, qt * BQ, a.T, a.hd);
    const int t = threadIdx.x;
    if (t < 2 * BQ) {
      const int q = qt * BQ + (t & (BQ - 1));
      rl = q < a.T ? (t < BQ ? lseg[q] : dlg[q]) : 0.f;
    }
    if (a.thr) {
      const int q = qt * BQ + (t >> 2), j = t & 3;
      rmw = (q < a.T && t0w + j < ntw) ? a.dmask[((long)bh * a.T + q) * ntw + t0w + j] : 0u;
    }
  };
  auto commit = [&]() {
    store64(smem + BWD_Q_OFF, rq);
    store64(smem + BWD_DO_OFF, rd);
    if (threadIdx.x < 2 * BQ) reinterpret_cast<float*>(smem + BWD_LD_OFF)[threadIdx.x] = rl;
    if (a.thr) reinterpret_cast<uint32_t*>(smem + BWD_MW_OFF)[threadIdx.x] = rmw;
  };
  issue(qt0);
  commit();
  __syncthreads();

  for (int qt = qt0; qt < nqt; ++qt) {
    const char* sQ = smem + BWD_Q_OFF;
    const char* sdO = smem + BWD_DO_OFF;
    // opaque per-iteration lane id: keeps the (loop-invariant) LDS addresses from being hoisted
    // into dozens of live VGPRs; they are recomputed with a few VALU ops instead.
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const int h32 = lane >> 5, l32 = lane & 31;
    const bool more = qt + 1 < nqt;
    if (more) issue(qt + 1);
    const int qbase = qt * BQ;
    char* myds = sdS + w * 32 * ROWB;  // this wave's 32 key rows of the dS^T image
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qsub0 = qbase + qs * 32;
      if (qsub0 + 31 < wave_kmin || wave_kmin >= a.T) {  // every query precedes every key: dS = 0
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qc = qs * 32 + 8 * g + 4 * h32;
          *reinterpret_cast<uint2*>(myds + lds_off(l32, qc >> 3) + (qc & 7) * 2) = make_uint2(0, 0);
        }
        continue;
      }
      f32x16 s = {0}, dp = {0};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_frag(sQ, qs * 32 + l32, ks * 2 + h32),
                                                    lds_row_frag(sK, 32 * w + l32, ks * 2 + h32), s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_frag(sdO, qs * 32 + l32, ks * 2 + h32), vf[ks], dp, 0, 0, 0);
      }
      // rows = queries qs*32 + (r&3) + 8(r>>2) + 4*h32 ; col = key (lane).  In place:
      // s <- dropped P (dV operand), dp <- dS = P * (dP~ * Z - delta).
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = qs * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
        const int q = qbase + ql;
        float p = fexp2(s[r] * a.scale_log2 - sL[ql]);
        if (mykey > q || q >= a.T) p = 0.f;
        float dpv = dp[r], pdrop = p;
        if (a.thr) {
          const float z = (sMW[ql * 4 + mw_col] >> mw_bit) & 1u ? a.dscale : 0.f;
          pdrop = p * z;
          dpv *= z;
        }
        s[r] = pdrop;
        dp[r] = p * (dpv - sL[BQ + ql]);
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pf = pack_frag(s, st);
        const bf16x8 dsf = pack_frag(dp, st);
        const int r0 = qs * 32 + 16 * st + 4 * h32;
        const int cb = 16 * ((lane >> 4) & 1);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sdO, r0, r0 + 8, cb, lane), pf, dv0, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sQ, r0, r0 + 8, cb, lane), dsf, dk0, 0, 0, 0);
        if constexpr (NKS > 2) {
          dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sdO, r0, r0 + 8, 32 + cb, lane), pf, dv1, 0, 0, 0);
          dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(sQ, r0, r0 + 8, 32 + cb, lane), dsf, dk1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // dS^T image row = key, 4 consecutive q per 8-byte write
        const int qc = qs * 32 + 8 * g + 4 * h32;
        *reinterpret_cast<uint2*>(myds + lds_off(l32, qc >> 3) + (qc & 7) * 2) =
            make_uint2(pack2(dp[4 * g], dp[4 * g + 1]), pack2(dp[4 * g + 2], dp[4 * g + 3]));
      }
    }
    __syncthreads();  // dS of all 128 keys in LDS; Q/dO tile no longer needed
    // dQ[64 q][64 d] = dS[64 q][128 keys] K[128 keys][64 d]: wave w owns the 32x32 output tile
    // (qs = w>>1, dblk = w&1) over all 128 keys -- no cross-wave reduction, one fp32 atomic per
    // element per workgroup (two 128-B row segments per wave-instruction).
    {
      const int qs = w >> 1, dblk = w & 1;
      if (dblk * 32 < a.hd && qbase + qs * 32 + 31 >= kb0) {
        f32x16 dq = {0};
        const int cb = 16 * ((lane >> 4) & 1);
#pragma unroll 2
        for (int kk = 0; kk < 8; ++kk) {
          const int kr0 = kk * 16 + 8 * h32;
          const bf16x8 af = lds_tr_frag(sdS, kr0, kr0 + 4, qs * 32 + cb, lane);
          dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, lds_tr_frag(sK, kr0, kr0 + 4, dblk * 32 + cb, lane), dq, 0, 0, 0);
        }
        const int d = dblk * 32 + l32;
        if (d < a.hd) {
          float* dqb = a.dq + ((long)b * a.T) * a.D + hh * a.hd + d;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = qbase + qs * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
            if (q < a.T) atomicAdd(dqb + (long)q * a.D, dq[r]);
          }
        }
      }
    }
    if (more) commit();
    __syncthreads();
  }

  // dK (scaled), dV -> dqkv K / V slots ; lane holds d = (r&3) + 8(r>>2) + 4*h32 (+32), key = lane
  const int lane = threadIdx.x & 63, h32 = lane >> 5;
  if (mykey < a.T) {
    const float sc = a.scale_log2 * 0.6931471805599453f;  // 1/sqrt(hd)
    bf16_t* krow = a.dqkv + ((long)b * a.T + mykey) * ld + a.D + hh * a.hd;
    bf16_t* vrow = krow + a.D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 8 * g + 4 * h32;
      if (d < a.hd) {
        *reinterpret_cast<uint2*>(krow + d) = make_uint2(pack2(dk0[4 * g] * sc, dk0[4 * g + 1] * sc),
                                                         pack2(dk0[4 * g + 2] * sc, dk0[4 * g + 3] * sc));
        *reinterpret_cast<uint2*>(vrow + d) = make_uint2(pack2(dv0[4 * g], dv0[4 * g + 1]),
                                                         pack2(dv0[4 * g + 2], dv0[4 * g + 3]));
      }
      if (32 + d < a.hd) {
        *reinterpret_cast<uint2*>(krow + 32 + d) = make_uint2(pack2(dk1[4 * g] * sc, dk1[4 * g + 1] * sc),
                                                              pack2(dk1[4 * g + 2] * sc, dk1[4 * g + 3] * sc));
        *reinterpret_cast<uint2*>(vrow + 32 + d) = make_uint2(pack2(dv1[4 * g], dv1[4 * g + 1]),
                                                              pack2(dv1[4 * g + 2], dv1[4 * g + 3]));
      }
    }
  }
}

// ------------------------------------------------------------------------------- backward, 256 keys
// Same algorithm, 8 waves = 256 keys per workgroup (1 workgroup / CU, 2 waves / SIMD): dQ of a
// query row is summed over T/256 instead of T/128 key blocks, halving the fp32 atomic bytes, which
// at ~1.3 TB/s chip-wide are this pass's floor (MI355X_MICROARCH 'Global float atomics').  The two
// waves that split a 32x32 dQ tile's 256 keys add their partials through LDS first.
// Per-element math: S accumulators start at -lse/c (p = exp2(c * S)), lse/delta/keep-words are read
// 4 rows per ds_read_b128, the causal mask runs only on diagonal tiles.
constexpr int KB2 = 256;
constexpr int B2_Q = 0;
constexpr int B2_DO = B2_Q + BQ * ROWB;             // 8 KiB
constexpr int B2_K = B2_DO + BQ * ROWB;             // 16 KiB
constexpr int B2_DS = B2_K + KB2 * ROWB;            // 48 KiB
constexpr int B2_L = B2_DS + KB2 * ROWB;            // 80 KiB: lse/c [64], delta [64] f32
constexpr int B2_MW = B2_L + 2 * BQ * 4;            // keep-words [8 cols][64 q] u32
constexpr int B2_P = B2_MW + 8 * BQ * 4;            // dQ partials [4 tiles][4][64 lanes][4] f32
constexpr int B2_SMEM = B2_P + 4 * 4 * 64 * 16;     // 99 KiB

// [rows][64 cols] bf16 tile -> LDS image (lds_off swizzle), NT threads, rows multiple of NT/8
template <int ROWS, int NT>
MG_DEVICE void load_rows(uint4 (&reg)[ROWS * 8 / NT], const bf16_t* base, long ld, int r0, int rows, int hd) {
#pragma unroll
  for (int i = 0; i < ROWS * 8 / NT; ++i) {
    const int idx = threadIdx.x + NT * i;
    const int row = idx >> 3, ch = idx & 7;
    const int r = r0 + row;
    reg[i] = (r < rows && ch * 8 < hd) ? ld16(base + (long)r * ld + ch * 8) : make_uint4(0, 0, 0, 0);
  }
}
template <int ROWS, int NT>
MG_DEVICE void store_rows(char* lds, const uint4 (&reg)[ROWS * 8 / NT]) {
#pragma unroll
  for (int i = 0; i < ROWS * 8 / NT; ++i) {
    const int idx = threadIdx.x + NT * i;
    *reinterpret_cast<uint4*>(lds + lds_off(idx >> 3, idx & 7)) = reg[i];
  }
}

// In place on one 32x32 (query rows x key lanes) tile: s <- dropped P (dV operand),
// dp <- dS = P * (dP~ * Z - delta).  Row r of the lane is query q0 + (r & 3) + 8 (r >> 2).
template <bool MASK>
MG_DEVICE void bwd_softmax_grad(f32x16& s, f32x16& dp, const float (&dl)[16], const uint32_t (&mwr)[16],
                                const AttnArgs& a, int mykey, int mw_bit, int q0) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float p = fexp2(s[r] * a.scale_log2);
    if constexpr (MASK) {
      // select, not a branch (a per-element if became an exec-mask branch per element)
      const int q = q0 + (r & 3) + 8 * (r >> 2);
      const bool kill = (mykey > q) | (q >= a.T);  // bitwise: no short-circuit branches
      p = kill ? 0.f : p;
    }
    float dpv = dp[r], pdrop = p;
    if (a.thr) {
      const float z = (mwr[r] >> mw_bit) & 1u ? a.dscale : 0.f;
      pdrop = p * z;
      dpv *= z;
    }
    s[r] = pdrop;
    dp[r] = p * (dpv - dl[r]);
  }
}

// bwd256 form: K is pre-scaled by c in LDS, so S' = Q (cK)^T - lse arrives in the log2 domain and
// p = exp2(S') needs no multiply.  Dropout keeps/zeroes with a sign-extended bit field (v_bfe_i32
// + v_and, no compare/select) and its 1/(1-p) is folded: into dS through one FMA, into dV at the
// store.  dS = P * (Z dP~ / (1-p) - delta); s <- Z P (dV operand, unscaled).
template <bool MASK>
MG_DEVICE void bwd_softmax_grad2(f32x16& s, f32x16& dp, const float (&dl)[16], const uint32_t (&mwr)[16],
                                 const AttnArgs& a, int mykey, int mw_bit, int q0) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float p = fexp2(s[r]);
    if constexpr (MASK) {
      const int q = q0 + (r & 3) + 8 * (r >> 2);
      const bool kill = (mykey > q) | (q >= a.T);
      p = kill ? 0.f : p;
    }
    // no dropout: every keep word is all ones (set when staged), dscale = 1
    const int keep = __builtin_amdgcn_sbfe((int)mwr[r], mw_bit, 1);  // 0 or -1
    s[r] = __int_as_float(__float_as_int(p) & keep);
    const float dpv = __int_as_float(__float_as_int(dp[r]) & keep);
    dp[r] = p * __builtin_fmaf(dpv, a.dscale, -dl[r]);
  }
}

template <int NKS>
__global__ __launch_bounds__(512, 1) void attn_bwd256_kernel(const AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x >> 6;
  const int bh = blockIdx.x % (a.B * a.H);
  const int kb = blockIdx.x / (a.B * a.H);  // key block 0 (sweeps every query) first
  const int b = bh / a.H, hh = bh % a.H;
  const int kb0 = kb * KB2;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  const bf16_t* Vg = Qg + 2 * a.D;
  const bf16_t* dOg = a.dout + (long)b * a.T * a.D + hh * a.hd;
  const float* lseg = a.lse + (long)bh * a.T;
  const float* dlg = a.delta + (long)bh * a.T;
  char* sK = smem + B2_K;
  char* sdS = smem + B2_DS;
  const float* sL = reinterpret_cast<const float*>(smem + B2_L);
  const uint32_t* sMW = reinterpret_cast<const uint32_t*>(smem + B2_MW);

  int mykey, wave_kmin;
  bf16x8 vf[4];
  {
    const int lane = threadIdx.x & 63, h32 = lane >> 5, l32 = lane & 31;
    mykey = kb0 + 32 * w + l32;
    wave_kmin = kb0 + 32 * w;
    uint4 rk[4];
    load_rows<KB2, 512>(rk, Kg, ld, kb0, a.T, a.hd);
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // K <- c K (see bwd_softmax_grad2); dQ is rescaled by ln 2
      float f[8];
      unpack8(rk[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= a.scale_log2;
      rk[i] = pack8(f);
    }
    store_rows<KB2, 512>(sK, rk);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d = ks * 16 + 8 * h32;
      const bool ok = mykey < a.T && d < a.hd;
      vf[ks] = __builtin_bit_cast(bf16x8, ok ? ld16(Vg + (long)mykey * ld + d) : make_uint4(0, 0, 0, 0));
    }
  }
  // this lane's dropout bit inside the forward's keep-words (see attn_fwd_kernel)
  const int mw_col = (w >> 1) * 2 + ((mykey >> 2) & 1);
  const int mw_el = ((mykey & 32) >> 1) | (mykey & 3) | (((mykey >> 3) & 3) << 2);  // fwd element
  const int mw_bit = 8 * (mw_el & 3) + (mw_el >> 2);  // its bit in the keep word (attn_fwd_kernel)
  const int ntw = 2 * ((a.T + 63) / 64);
  const int t0w = (kb0 / 64) * 2;

  f32x16 dk0 = {0}, dk1 = {0}, dv0 = {0}, dv1 = {0};
  const int qt0 = kb0 / BQ;
  const int nqt = (a.T + BQ - 1) / BQ;

  uint4 rq[1], rd[1];
  float rl = 0.f;
  uint32_t rmw = 0xffffffffu;  // no dropout: every key kept
  auto issue = [&](int qt) {
    load_rows<BQ, 512>(rq, Qg, ld, qt * BQ, a.T, a.hd);
    load_rows<BQ, 512>(rd, dOg, a.D, qt * BQ, a.T, a.hd);
    const int t = threadIdx.x;
    if (t < 2 * BQ) {
      const int q = qt * BQ + (t & (BQ - 1));
      rl = q < a.T ? (t < BQ ? -lseg[q] : dlg[q]) : 0.f;  // -lse: the S init (K holds c K)
    }
    if (a.thr) {  // word j of query row q -> sMW[j * 64 + q]
      const int q = qt * BQ + (t & 63), j = t >> 6;
      rmw = (q < a.T && t0w + j < ntw) ? a.dmask[((long)bh * a.T + q) * ntw + t0w + j] : 0u;
    }
  };
  auto commit = [&]() {
    store_rows<BQ, 512>(smem + B2_Q, rq);
    store_rows<BQ, 512>(smem + B2_DO, rd);
    if (threadIdx.x < 2 * BQ) reinterpret_cast<float*>(smem + B2_L)[threadIdx.x] = rl;
    reinterpret_cast<uint32_t*>(smem + B2_MW)[threadIdx.x] = rmw;
  };
  issue(qt0);
  commit();
  __syncthreads();

  for (int qt = qt0; qt < nqt; ++qt) {
    const char* sQ = smem + B2_Q;
    const char* sdO = smem + B2_DO;
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));  // recomputed per tile: keeps the offsets below out of the loop state
    const int h32 = lane >> 5, l32 = lane & 31;
    const bool more = qt + 1 < nqt;
    if (more) issue(qt + 1);
    const int qbase = qt * BQ;
    char* myds = sdS + w * 32 * ROWB;
    // per-lane LDS offsets for this tile (row bases of 16-row multiples go into immediates):
    // row reads of row l32, chunk 2 ks + h32; transposed reads rows 4 h32 + q (+8), cols cb + 4p (+32)
    const char* sKw = sK + w * 32 * ROWB;
    int ro[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) ro[ks] = lds_off(l32, 2 * ks + h32);
    const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
    const int ta0 = tr_off(4 * h32 + trq, trc), tb0 = tr_off(8 + 4 * h32 + trq, trc);
    const int ta1 = tr_off(4 * h32 + trq, 32 + trc), tb1 = tr_off(8 + 4 * h32 + trq, 32 + trc);
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qsub0 = qbase + qs * 32;
      if (qsub0 + 31 < wave_kmin || wave_kmin >= a.T) {  // every query precedes every key: dS = 0
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qc = qs * 32 + 8 * g + 4 * h32;
          *reinterpret_cast<uint2*>(myds + lds_off(l32, qc >> 3) + (qc & 7) * 2) = make_uint2(0, 0);
        }
        continue;
      }
      // row constants of this lane's 16 rows (4 consecutive rows per float4)
      float lr[16], dl[16];
      uint32_t mwr[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q4 = qs * 32 + 8 * g + 4 * h32;
        const float4 x = *reinterpret_cast<const float4*>(sL + q4);
        const float4 y = *reinterpret_cast<const float4*>(sL + BQ + q4);
        lr[4 * g] = x.x; lr[4 * g + 1] = x.y; lr[4 * g + 2] = x.z; lr[4 * g + 3] = x.w;
        dl[4 * g] = y.x; dl[4 * g + 1] = y.y; dl[4 * g + 2] = y.z; dl[4 * g + 3] = y.w;
        {
          const uint4 m4 = *reinterpret_cast<const uint4*>(sMW + mw_col * 64 + q4);
          mwr[4 * g] = m4.x; mwr[4 * g + 1] = m4.y; mwr[4 * g + 2] = m4.z; mwr[4 * g + 3] = m4.w;
        }
      }
      f32x16 s, dp = {0};
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = lr[r];  // S' = Q K^T - lse/c
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sQ + qs * 32 * ROWB, ro[ks]),
                                                    lds_row_at(sKw, ro[ks]), s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sdO + qs * 32 * ROWB, ro[ks]), vf[ks], dp, 0, 0, 0);
      }
      // rows = queries qs*32 + (r&3) + 8(r>>2) + 4*h32 ; col = key (lane).  In place:
      // s <- dropped P (dV operand), dp <- dS = P * (dP~ * Z - delta).
      // wave-uniform: only diagonal / past-T tiles pay for the causal mask
      if (wave_kmin + 31 > qsub0 || qsub0 + 31 >= a.T)
        bwd_softmax_grad2<true>(s, dp, dl, mwr, a, mykey, mw_bit, qsub0 + 4 * h32);
      else
        bwd_softmax_grad2<false>(s, dp, dl, mwr, a, mykey, mw_bit, qsub0 + 4 * h32);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pf = pack_frag(s, st);
        const bf16x8 dsf = pack_frag(dp, st);
        const int rb = (qs * 32 + 16 * st) * ROWB;  // 16-row aligned: an immediate
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sdO + rb, ta0, tb0), pf, dv0, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sQ + rb, ta0, tb0), dsf, dk0, 0, 0, 0);
        if constexpr (NKS > 2) {
          dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sdO + rb, ta1, tb1), pf, dv1, 0, 0, 0);
          dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sQ + rb, ta1, tb1), dsf, dk1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // dS^T image row = key, 4 consecutive q per 8-byte write
        const int qc = qs * 32 + 8 * g + 4 * h32;
        *reinterpret_cast<uint2*>(myds + lds_off(l32, qc >> 3) + (qc & 7) * 2) =
            make_uint2(pack2(dp[4 * g], dp[4 * g + 1]), pack2(dp[4 * g + 2], dp[4 * g + 3]));
      }
    }
    __syncthreads();  // dS of all 256 keys in LDS
    // dQ[64 q][64 d] = dS[64 q][256 keys] K[256 keys][64 d]: 32x32 output tile (qs, dblk) = w & 3,
    // key half kh = w >> 2; the kh = 1 wave hands its partial to the kh = 0 wave through LDS.
    const int tile = w & 3, kh = w >> 2;
    const int qs = tile >> 1, dblk = tile & 1;
    const bool act1 = dblk * 32 < a.hd && qbase + qs * 32 + 31 >= kb0 + 128 && kb0 + 128 < a.T;
    const bool act0 = dblk * 32 < a.hd && qbase + qs * 32 + 31 >= kb0;
    f32x16 dq = {0};
    if (kh ? act1 : act0) {
      // rows kh*128 + 16 kk + 8 h32 + q (+4): the 16 kk part is an immediate
      const int da = tr_off(8 * h32 + trq, qs * 32 + trc), db = tr_off(8 * h32 + 4 + trq, qs * 32 + trc);
      const int ko = tr_off(8 * h32 + trq, dblk * 32 + trc), ko4 = tr_off(8 * h32 + 4 + trq, dblk * 32 + trc);
      const char* sdSh = sdS + kh * 128 * ROWB;
      const char* sKh = sK + kh * 128 * ROWB;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sdSh + kk * 16 * ROWB, da, db),
                                                     lds_tr_at(sKh + kk * 16 * ROWB, ko, ko4), dq, 0, 0, 0);
    }
    float* part = reinterpret_cast<float*>(smem + B2_P) + tile * 4 * 64 * 4;
    if (kh == 1 && act1) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(part + (g * 64 + lane) * 4) =
            f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
    }
    __syncthreads();
    if (kh == 0 && act0) {
      if (act1) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(part + (g * 64 + lane) * 4);
          dq[4 * g] += x[0]; dq[4 * g + 1] += x[1]; dq[4 * g + 2] += x[2]; dq[4 * g + 3] += x[3];
        }
      }
      // this key block's partial: plain stores (rows q >= kb0 are all written by this workgroup;
      // attn_dq_finalize sums the partials of key blocks kb0 <= q), no atomics, no memset
      const int d = dblk * 32 + l32;
      if (d < a.hd) {
        // row q0 + (r & 3) + 8 (r >> 2): one 64-bit base per lane, then uniform row strides
        const int q0 = qbase + qs * 32 + 4 * h32;
        float* dqb = a.dq + kb * a.dq_part + ((long)b * a.T + q0) * a.D + hh * a.hd + d;
        const long rs = a.D;
        if (qbase + BQ <= a.T) {  // whole tile inside the sequence: no per-row checks
#pragma unroll
          for (int r = 0; r < 16; ++r) dqb[((r & 3) + 8 * (r >> 2)) * rs] = dq[r];
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (q0 + (r & 3) + 8 * (r >> 2) < a.T) dqb[((r & 3) + 8 * (r >> 2)) * rs] = dq[r];
        }
      }
    }
    if (more) commit();
    __syncthreads();
  }

  const int lane = threadIdx.x & 63, h32 = lane >> 5;
  if (mykey < a.T) {
    const float sc = a.scale_log2 * 0.6931471805599453f;  // 1/sqrt(hd)
    const float vs = a.thr ? a.dscale : 1.f;                // dropout keep scale, folded (see above)
    bf16_t* krow = a.dqkv + ((long)b * a.T + mykey) * ld + a.D + hh * a.hd;
    bf16_t* vrow = krow + a.D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 8 * g + 4 * h32;
      if (d < a.hd) {
        *reinterpret_cast<uint2*>(krow + d) = make_uint2(pack2(dk0[4 * g] * sc, dk0[4 * g + 1] * sc),
                                                         pack2(dk0[4 * g + 2] * sc, dk0[4 * g + 3] * sc));
        *reinterpret_cast<uint2*>(vrow + d) = make_uint2(pack2(dv0[4 * g] * vs, dv0[4 * g + 1] * vs),
                                                         pack2(dv0[4 * g + 2] * vs, dv0[4 * g + 3] * vs));
      }
      if (32 + d < a.hd) {
        *reinterpret_cast<uint2*>(krow + 32 + d) = make_uint2(pack2(dk1[4 * g] * sc, dk1[4 * g + 1] * sc),
                                                              pack2(dk1[4 * g + 2] * sc, dk1[4 * g + 3] * sc));
        *reinterpret_cast<uint2*>(vrow + 32 + d) = make_uint2(pack2(dv1[4 * g] * vs, dv1[4 * g + 1] * vs),
                                                              pack2(dv1[4 * g + 2] * vs, dv1[4 * g + 3] * vs));
      }
    }
  }
}

// dqkv Q slot = bf16(scale * sum of the dQ partials).  part = 0: one atomic accumulator;
// otherwise partial kb (stride part) holds key block kb's contribution for rows t >= kb * KB2.
__global__ __launch_bounds__(256) void attn_dq_finalize_kernel(const float* __restrict__ dq,
                                                               bf16_t* __restrict__ dqkv, long rows,
                                                               int D, int T, long part, float sc) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over rows * D/8
  const long n8 = rows * (D / 8);
  if (i >= n8) return;
  const long r = i / (D / 8);
  const int c = (int)(i % (D / 8)) * 8;
  const int np = part ? (int)(r % T) / KB2 + 1 : 1;
  float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
  for (int k = 0; k < np; ++k) {
    const float* src = dq + k * part + r * D + c;
    const float4 y0 = *reinterpret_cast<const float4*>(src), y1 = *reinterpret_cast<const float4*>(src + 4);
    x0.x += y0.x; x0.y += y0.y; x0.z += y0.z; x0.w += y0.w;
    x1.x += y1.x; x1.y += y1.y; x1.z += y1.z; x1.w += y1.w;
  }
  const float f[8] = {x0.x * sc, x0.y * sc, x0.z * sc, x0.w * sc, x1.x * sc, x1.y * sc, x1.z * sc, x1.w * sc};
  st16(dqkv + r * 3L * D + c, pack8(f));
}

// =============================================================================== decode
// One new query per sequence attending to a KV cache held as qkv rows [B, Tmax, 3D] (the prefill
// writes its qkv GEMM output straight into it).  Appends this step's K/V at row `pos`, then
// softmax over keys 0..pos.  grid = B*H, 256 threads; scores live in LDS (Tmax floats).
__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16_t* __restrict__ qkv_new,
                                                          bf16_t* __restrict__ cache,
                                                          bf16_t* __restrict__ out, int H, int hd,
                                                          int D, long Tmax, int pos,
                                                          const int* __restrict__ pos_dev,
                                                          float scale_log2) {
  if (pos_dev) pos = min(max(*pos_dev, 0), (int)Tmax - 1);  // hipGraph decode: position in device memory
  extern __shared__ __attribute__((aligned(16))) float dsm[];  // [64 q][Tmax scores][32*64 acc][8]
  float* qs = dsm;
  float* sc = dsm + 64;
  float* acc = sc + ((Tmax + 3) & ~3L);
  float* red = acc + 32 * 64;
  const int b = blockIdx.x / H, hh = blockIdx.x % H;
  const long ld = 3L * D;
  const bf16_t* qrow = qkv_new + (long)b * ld + hh * hd;
  bf16_t* cb = cache + (long)b * Tmax * ld;
  for (int i = threadIdx.x; i < 2 * hd; i += 256) {
    const int which = i / hd, d = i % hd;
    cb[(long)pos * ld + (long)D * (1 + which) + hh * hd + d] = qrow[(long)D * (1 + which) + d];
  }
  for (int d = threadIdx.x; d < hd; d += 256) qs[d] = bf2f(qrow[d]);
  __syncthreads();
  const int L = pos + 1;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < L; j += 256) {
    const bf16_t* kr = (j == pos) ? qrow + D : cb + (long)j * ld + D + hh * hd;
    float s = 0.f;
    for (int d = 0; d < hd; d += 8) {
      float k8[8];
      unpack8(ld16(kr + d), k8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qs[d + e] * k8[e];
    }
    s *= scale_log2;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max<4>(mx, red);
  float sm = 0.f;
  for (int j = threadIdx.x; j < L; j += 256) {
    const float p = fexp2(sc[j] - mx);
    sc[j] = p;
    sm += p;
  }
  sm = block_sum<4>(sm, red + 4);
  __syncthreads();
  // P V: 32 key groups x 8 lanes of 8 dims (16-byte V loads), folded through LDS
  const int grp = threadIdx.x >> 3, d8 = (threadIdx.x & 7) * 8;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (d8 < hd) {
    for (int j = grp; j < L; j += 32) {
      const bf16_t* vr = (j == pos) ? qrow + 2 * D : cb + (long)j * ld + 2 * D + hh * hd;
      float v8[8];
      unpack8(ld16(vr + d8), v8);
      const float p = sc[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += p * v8[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[grp * 64 + d8 + e] = o[e];
  __syncthreads();
  if (threadIdx.x < hd) {
    float v = 0.f;
#pragma unroll 8
    for (int g = 0; g < 32; ++g) v += acc[g * 64 + threadIdx.x];
    out[(long)b * D + hh * hd + threadIdx.x] = f2bf(v / sm);
  }
}

}  // namespace

namespace mg {

void attention_decode(const bf16_t* qkv_new, bf16_t* cache, bf16_t* out, int B, int H, int hd,
                      long Tmax, int pos, hipStream_t stream, const int* pos_dev) {
  const size_t smem = sizeof(float) * (64 + ((Tmax + 3) & ~3L) + 32 * 64 + 8);
  attn_decode_kernel<<<B * H, 256, smem, stream>>>(qkv_new, cache, out, H, hd, H * hd, Tmax, pos,
                                                   pos_dev, 1.4426950408889634f / sqrtf((float)hd));
}

static int g_attn_bwd_variant = 0;  // 0 auto (256-key blocks), 1 force 128-key blocks

static AttnArgs make_args(int B, int T, int H, int hd, float p, uint64_t seed) {
  AttnArgs a{};
  a.B = B; a.T = T; a.H = H; a.hd = hd; a.D = H * hd;
  a.scale_log2 = 1.4426950408889634f / sqrtf((float)hd);
  a.seed = seed;
  a.sofs = graph_seed_ofs();
  {  // host copy of mix32: per-launch key for the forward's dropout hash
    auto mix = [](uint32_t x) {
      x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
      return x;
    };
    a.seed_key = mix((uint32_t)seed) ^ mix((uint32_t)(seed >> 32) + 0x9E3779B9u);
  }
  // 8-bit dropout threshold (as FlashAttention does): effective p = thr / 256
  int thr = p > 0.f ? (int)lrintf(p * 256.f) : 0;
  if (p > 0.f) thr = thr < 1 ? 1 : (thr > 255 ? 255 : thr);
  a.thr = (uint32_t)thr;
  a.dscale = thr ? 256.f / (256.f - (float)thr) : 1.f;
  a.kadd = (uint32_t)(thr <= 128 ? 128 - thr : 256 - thr) * 0x01010101u;
  return a;
}

void attention_set_bwd_variant(int v) { g_attn_bwd_variant = v; }

// number of dQ partial buffers attention_bwd needs (the 256-key kernel writes one per key block)
int attention_bwd_keyblocks(int T) { return (g_attn_bwd_variant != 1 && T > 128) ? cdiv(T, KB2) : 1; }

size_t attention_dropout_mask_words(int B, int T, int H) {
  return (size_t)B * H * T * 2 * ((T + 63) / 64);
}

void attention_fwd(const bf16_t* qkv, bf16_t* out, float* lse, uint32_t* dmask, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream) {
  AttnArgs a = make_args(B, T, H, hd, p, seed);
  a.qkv = qkv; a.out = out; a.lse = lse; a.dmask = dmask;
  if (a.thr && !dmask) a.thr = 0;
  const int grid = cdiv(T, 128) * B * H;
  if (hd > 32) attn_fwd_kernel<4><<<grid, 256, 0, stream>>>(a);
  else if (hd > 16) attn_fwd_kernel<2><<<grid, 256, 0, stream>>>(a);
  else attn_fwd_kernel<1><<<grid, 256, 0, stream>>>(a);
}

void attention_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse,
                   const uint32_t* dmask, float* delta, float* dq, bf16_t* dqkv, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream) {
  AttnArgs a = make_args(B, T, H, hd, p, seed);
  a.qkv = qkv; a.out = dqkv; a.lse = const_cast<float*>(lse); a.dout = dout; a.delta = delta;
  a.dq = dq; a.dqkv = dqkv; a.dmask = const_cast<uint32_t*>(dmask);
  if (a.thr && !dmask) a.thr = 0;
  const long nchunks = (long)B * T * H * hd / 8;
  attn_bwd_pre_kernel<<<cdiv(nchunks, 256), 256, 0, stream>>>(dout, out, delta, B, T, H, hd, H * hd);
  const bool blk256 = g_attn_bwd_variant != 1 && T > 128;
  a.dq_part = blk256 ? (long)B * T * H * hd : 0;
  if (!blk256) hipMemsetAsync(dq, 0, sizeof(float) * (size_t)B * T * H * hd, stream);
  if (blk256) {  // 256-key blocks, dQ partials per key block
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)attn_bwd256_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, B2_SMEM);
      hipFuncSetAttribute((const void*)attn_bwd256_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, B2_SMEM);
      hipFuncSetAttribute((const void*)attn_bwd256_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, B2_SMEM);
      attr = true;
    }
    const int grid = cdiv(T, KB2) * B * H;
    if (hd > 32) attn_bwd256_kernel<4><<<grid, 512, B2_SMEM, stream>>>(a);
    else if (hd > 16) attn_bwd256_kernel<2><<<grid, 512, B2_SMEM, stream>>>(a);
    else attn_bwd256_kernel<1><<<grid, 512, B2_SMEM, stream>>>(a);
  } else {
    const int grid = cdiv(T, 128) * B * H;
    if (hd > 32) attn_bwd_kernel<4><<<grid, 256, BWD_SMEM, stream>>>(a);
    else if (hd > 16) attn_bwd_kernel<2><<<grid, 256, BWD_SMEM, stream>>>(a);
    else attn_bwd_kernel<1><<<grid, 256, BWD_SMEM, stream>>>(a);
  }
  const long n8 = (long)B * T * (H * hd / 8);
  // dQ = dS K / sqrt(hd); the 256-key kernel multiplied by c K = log2(e) K / sqrt(hd) -> ln 2
  const float dq_scale = blk256 ? 0.6931471805599453f : 1.f / sqrtf((float)hd);
  attn_dq_finalize_kernel<<<cdiv(n8, 256), 256, 0, stream>>>(dq, dqkv, (long)B * T, H * hd, T,
                                                             a.dq_part, dq_scale);
}

}  // namespace mg
