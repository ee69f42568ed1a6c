// Causal flash attention backward for training on gfx950 (CDNA4, MI355X).  (Dropout keep bits and
// the forward: attention_fwd.hip; decode: attention.hip.)
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

// =============================================================================== backward
// delta[(b*H + h)*T + t] = sum_d dO * O.  One lane per 16-byte chunk (8 elements) of a head row,
// lanes of consecutive chunks/heads/tokens read contiguous memory; the ceil(hd/8) lanes of a
// head row are reduced with xor-shuffles (groups padded to a power of two).
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ out,
                                                           float* __restrict__ delta, int BT, int T,
                                                           int H, int hd, int lg, int* __restrict__ work) {
  // thread -> (row bt, head h, chunk c < cpr = 2^lg): cpr = chunks per head row rounded up to a
  // power of two; 32-bit index arithmetic (B*T*H*cpr < 2^31 is checked on the host)
  const int cpr = 1 << lg;
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i == 0 && work) *work = 0;  // attn_bwd64_kernel's item counter, for the launch after this one
  const int c = (int)(i & (cpr - 1));
  const unsigned rh = i >> lg;
  const int hh = (int)(rh % (unsigned)H);
  const int bt = (int)(rh / (unsigned)H);
  float s = 0.f;
  if (bt < BT && c * 8 < hd) {
    const long e = bt * H * hd + (long)hh * hd + c * 8;
    float x[8], y[8];
    unpack8(ld16(dout + e), x);
    unpack8(ld16(out + e), y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
  for (int o = 1; o < cpr; o <<= 1) s += __shfl_xor(s, o, 64);
  if (bt < BT && c == 0) {
    const int t = (int)(bt % T), b = (int)(bt / T);
    delta[((long)b * H + hh) * T + t] = s;
  }
}

// queries per backward tile: 128 in key-block mode at hd 33..64 (two barriers per 128 queries, and
// as many 32x32 dQ tiles as waves: no split-key dQ hand-off in LDS), else 64
template <int NKS, bool PERSIST>
constexpr int bwd_bq() { return (!PERSIST && (NKS == 3 || NKS == 4)) ? 128 : 64; }

// In place on one 32x32 (query rows x key lanes) tile: s <- dropped P (dV operand), dp <- dS / dscale.
// K is pre-scaled by c in LDS, so S' = Q (cK)^T - lse arrives in the log2 domain and p = exp2(S').
// Dropout keeps/zeroes with a sign-extended bit field; its 1/(1-p) = dscale is taken out of dS:
// dS = P (Z dP~ dscale - delta) = dscale (ZP dP~ - P delta'), delta' = delta / dscale (staged so),
// and dscale goes into the dK / dQ output scales.  Per element: exp2, bfe, and, mul, fma (was bfe,
// two ands, fma, mul): 1,250 -> 1,227 us at B = 128.  The same with v_pk_mul / v_pk_fma per row
// pair measured 1,300 us (256 VGPRs, spills: pairs need aligned registers).
template <bool MASK>
MG_DEVICE void bwd_softmax_grad(f32x16& s, f32x16& dp, const float (&dl)[16], const uint32_t (&mwr)[16],
                                int T, int mykey, int mw_bit, int q0) {
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    float p[2], pd[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      p[u] = fexp2(s[r + u]);
      if constexpr (MASK) {
        const int q = q0 + ((r + u) & 3) + 8 * ((r + u) >> 2);
        const bool kill = (mykey > q) | (q >= T);  // bitwise: no short-circuit branches
        p[u] = kill ? 0.f : p[u];
      }
      // no dropout: every keep word is all ones (set when staged), dscale = 1.  One v_bfe_i32 (the
      // builtin became and + compare + select)
      int keep;
      asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(keep) : "v"(mwr[r + u]), "v"(mw_bit));
      pd[u] = __int_as_float(__float_as_int(p[u]) & keep);
      s[r + u] = pd[u];
    }
    dp[r] = __builtin_fmaf(pd[0], dp[r], -(p[0] * dl[r]));
    dp[r + 1] = __builtin_fmaf(pd[1], dp[r + 1], -(p[1] * dl[r + 1]));
  }
}

// Row r of bwd_softmax_grad<false> given p = exp2(S'[r]) (attn_bwd64_kernel's pinned schedule puts
// one beside each MFMA, with the next row's exp2 issued in the same slot: two independent chains
// instead of one 5-deep one per slot); the same operations, so the same results.
MG_DEVICE void bwd_softmax_one(f32x16& s, f32x16& dp, const float (&dl)[16], const uint32_t (&mwr)[16],
                               int mw_bit, int r, float p) {  // p = fexp2(s[r]), computed ahead
  // v_bfe_i32 through the builtin: an asm statement here cost an s_nop per element (hipcc pads
  // one state after every asm before a VALU reading its output)
  const int keep = __builtin_amdgcn_sbfe((int)mwr[r], mw_bit, 1);
  const float pd = __int_as_float(__float_as_int(p) & keep);
  s[r] = pd;
  dp[r] = __builtin_fmaf(pd, dp[r], -(p * dl[r]));
}

// Staging of a [ROWS][NH * 64] bf16 tile (columns >= hd zero) into NH 64-column LDS images.
// Addresses are recomputed from threadIdx at each use (a few VALU ops): holding them across the
// kernel cost the backward its last free registers.
template <int ROWS, int NH, int NT>
struct Stager {
  static constexpr int N = ROWS * 8 * NH / NT;  // 16-byte chunks per thread
  static MG_DEVICE void load(uint4 (&reg)[N], const bf16_t* base, long ld, int r0, int rows, int hd) {
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int rem = idx % (ROWS * 8);
      const int r = r0 + (rem >> 3), col = (idx / (ROWS * 8)) * 64 + (rem & 7) * 8;
      reg[c] = (r < rows && col < hd) ? ld16(base + (long)r * ld + col) : make_uint4(0, 0, 0, 0);
    }
  }
  // per-thread byte offsets of its chunks from a tile's first row (computed once per kernel)
  static MG_DEVICE void offsets(uint32_t (&off)[N], long ld) {
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int rem = idx % (ROWS * 8);
      off[c] = (uint32_t)(((rem >> 3) * ld + (idx / (ROWS * 8)) * 64 + (rem & 7) * 8) * 2);
    }
  }
  // buffer loads through one descriptor per tile (base = the tile's first row, extent = the rest
  // of the tensor): no per-lane bounds branches or 64-bit address math per tile.  Rows past the
  // sequence read the next sequence's (finite) rows, past the tensor zeros; columns past hd read
  // the neighbouring head.  Callers make both harmless (attn_bwd_kernel: masked rows, zero K / V
  // columns past hd).
  static MG_DEVICE void load_buf(uint4 (&reg)[N], const bf16_t* tensor, uint64_t total, uint64_t origin,
                                 const uint32_t (&off)[N]) {
    const __amdgpu_buffer_rsrc_t d = kv_rsrc(tensor, total, origin);
#pragma unroll
    for (int c = 0; c < N; ++c) reg[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(d, off[c], 0, 0));
  }
  static MG_DEVICE void store(char* lds, const uint4 (&reg)[N]) {
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int rem = idx % (ROWS * 8);
      *reinterpret_cast<uint4*>(lds + (idx / (ROWS * 8)) * ROWS * ROWB + lds_off(rem >> 3, rem & 7)) = reg[c];
    }
  }
};

// Transpose-reduce over the 32 lanes of each half-wave: each step halves the values a lane keeps
// (the lane's bit M picks the half) and adds its partner's copy of that half, so a lane ends with
// NV / 32 sums, value index NV / 32 * (lane & 31) + j for v[j] -- 31 NV / 32 shuffles instead of
// 5 NV for a full butterfly per value.
template <int M, int C, int NV>
MG_DEVICE void tr_reduce32(float (&v)[NV], int lane) {
  const bool hi = lane & M;
#pragma unroll
  for (int i = 0; i < C / 2; ++i) {
    const float send = hi ? v[i] : v[i + C / 2];
    const float keep = hi ? v[i + C / 2] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
  if constexpr (M > 1) tr_reduce32<M / 2, C / 2, NV>(v, lane);
}

// Key-block-parallel backward, one workgroup per (b, h) sweeping its key blocks in order.
//  * KW waves = KB = 32 KW keys per block (K pre-scaled by log2(e)/sqrt(hd) in LDS); each wave
//    keeps its 32 keys' V rows (the dP~ B operand) and dK^T / dV^T accumulators (keys on the lane)
//    in registers across the block's query sweep.
//  * per 64-query tile (Q, dO, lse, delta, keep-words staged in LDS, the next tile prefetched in
//    VGPRs): S and dP with the key on the lane, P and dS in registers feed dV^T += dO^T P and
//    dK^T += Q^T dS directly (transposed reads of Q / dO); dS^T goes through LDS once for
//    dQ = dS K (the waves split the 32x32 dQ tiles and, where there are more waves than tiles,
//    the keys; partial tiles meet in LDS).
//  * dQ of a query tile is summed over the key blocks in a fp32 buffer that only this workgroup
//    touches (the first block stores, later ones read-add-store; each element always by the
//    same lane, so program order is the only ordering needed) and written as bf16 into dqkv by
//    the last block that reaches the tile: no per-key-block partial buffers, no finalize pass.
//  * attention dropout: the forward's keep bits (attn_dropmask_kernel), one word per query and
//    32-key half tile, staged BQ queries x KW words per tile.
//  * BQ = 128 queries per tile (key-block mode, hd <= 64): the dS^T image is two 64-query halves.
// (The round-4 timing-only ablations of this kernel -- outputs wrong on purpose -- live outside the
// production source: bench/dev/attn_ablations.patch, applied to a scratch copy by scripts/build_variant.sh.)
template <int NKS, int KW, bool PERSIST>
__global__ __launch_bounds__(64 * KW, 1) void attn_bwd_kernel(const AttnArgs a) {
  constexpr int BQ = bwd_bq<NKS, PERSIST>();
  constexpr int NQS = BQ / 32;                   // 32-query subtiles per tile
  constexpr int NH = (NKS + 3) / 4, NO = (NKS + 1) / 2;
  constexpr int NT = 64 * KW, KB = 32 * KW;
  constexpr int HQ = BQ * ROWB, HK = KB * ROWB;  // one 64-column half of a Q / K image
  constexpr int TILES = NQS * NO;                // 32x32 dQ tiles of a query tile
  constexpr int KSPLIT = KW >= TILES ? KW / TILES : 1;
  constexpr int OFF_Q = 0, OFF_DO = OFF_Q + NH * HQ, OFF_K = OFF_DO + NH * HQ;
  constexpr int OFF_DS = OFF_K + NH * HK, OFF_L = OFF_DS + (BQ / 64) * KB * ROWB;
  constexpr int OFF_MW = OFF_L + 2 * BQ * 4, OFF_P = OFF_MW + KW * BQ * 4;
  constexpr int OFF_PV = OFF_P + (KSPLIT > 1 ? (KSPLIT - 1) * TILES * 64 * 16 * 4 : 0);
  static_assert(BQ == 64 || (KSPLIT == 1 && !PERSIST), "BQ 128: key-block mode, no split-key dQ");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x >> 6;
  const int BH = a.B * a.H;
  const int bh = blockIdx.x % BH;
  const int b = bh / a.H, hh = bh % a.H;
  const long ld = 3L * a.D;
  const bf16_t* Qg = a.qkv + (long)b * a.T * ld + hh * a.hd;
  const bf16_t* Kg = Qg + a.D;
  const bf16_t* Vg = Qg + 2 * a.D;
  const bf16_t* dOg = a.dout + (long)b * a.T * a.D + hh * a.hd;
  const float* lseg = a.lse + (long)bh * a.T;
  const float* dlg = a.delta + (long)bh * a.T;
  char* sK = smem + OFF_K;
  char* sdS = smem + OFF_DS;
  const float* sL = reinterpret_cast<const float*>(smem + OFF_L);
  const uint32_t* sMW = reinterpret_cast<const uint32_t*>(smem + OFF_MW);
  const int ntw = 2 * ((a.T + 63) / 64);
  const int nqt = (a.T + BQ - 1) / BQ;
  const int nkb = (a.T + KB - 1) / KB;
  const float dq_scale = 0.6931471805599453f * a.dscale;  // dQ = dscale dS' (c K) ln 2 = dS K / sqrt(hd)
  const float ddl = 1.f / a.dscale;                         // delta' = delta / dscale (bwd_softmax_grad)

  using stq = Stager<BQ, NH, NT>;
  using stk = Stager<KB, NH, NT>;

  // this wave's dQ tiles: (tile, key split); tiles are (q-subtile qs, 32-column block n)
  const int my_split = KSPLIT > 1 ? w / TILES : 0;
  constexpr int KSPAN = KB / KSPLIT;  // keys per split (a multiple of 16)
  constexpr int NTW = KSPLIT > 1 ? 1 : (TILES + KW - 1) / KW;  // dQ tiles per wave
  const int tt0 = KSPLIT > 1 ? w % TILES : w;
  constexpr int TSTEP = KSPLIT > 1 ? TILES : KW;

  // persistent mode (dq_part == 0): this workgroup sweeps every key block of its (b, h); partial
  // mode: workgroup = one key block (heaviest first), its dQ contribution stored as partial kb
  constexpr bool part = !PERSIST;
  const int kb_lo = part ? blockIdx.x / BH : 0, kb_hi = part ? kb_lo + 1 : nkb;
  for (int kb = kb_lo; kb < kb_hi; ++kb) {
    const int kb0 = kb * KB;
    int mykey, wave_kmin;
    bf16x8 vf[NKS];  // this wave's 32 keys' V rows: the B operand of dP~ = dO V^T
    {
      const int lane = threadIdx.x & 63, h32 = lane >> 5, l32 = lane & 31;
      mykey = kb0 + 32 * w + l32;
      wave_kmin = kb0 + 32 * w;
      uint4 rk[Stager<KB, NH, NT>::N];
      stk::load(rk, Kg, ld, kb0, a.T, a.hd);
#pragma unroll
      for (int i = 0; i < Stager<KB, NH, NT>::N; ++i) {  // K <- c K (see bwd_softmax_grad)
        float f[8];
        unpack8(rk[i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= a.scale_log2;
        rk[i] = pack8(f);
      }
      __syncthreads();  // the previous block's readers of sK are done
      stk::store(sK, rk);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int d = ks * 16 + 8 * h32;
        const bool ok = mykey < a.T && d < a.hd;
        vf[ks] = __builtin_bit_cast(bf16x8, ok ? ld16(Vg + (long)mykey * ld + d) : make_uint4(0, 0, 0, 0));
      }
    }
    // this lane's dropout bit inside the keep words (attn_dropmask_kernel layout)
    const int mw_col = (w >> 1) * 2 + ((mykey >> 2) & 1);
    const int mw_el = ((mykey & 32) >> 1) | (mykey & 3) | (((mykey >> 3) & 3) << 2);
    const int mw_bit = drop_bit(mw_el);
    const int t0w = (kb0 / 64) * 2;

    f32x16 dk[NO], dv[NO];
#pragma unroll
    for (int n = 0; n < NO; ++n) {
      dk[n] = f32x16{0};
      dv[n] = f32x16{0};
    }
    const int qt0 = kb0 / BQ;

    uint4 rq[Stager<BQ, NH, NT>::N], rd[Stager<BQ, NH, NT>::N];
    uint32_t oq[Stager<BQ, NH, NT>::N], od[Stager<BQ, NH, NT>::N];
    stq::offsets(oq, ld);
    stq::offsets(od, a.D);
    const uint64_t q_total = (uint64_t)a.B * a.T * ld * 2, do_total = (uint64_t)a.B * a.T * a.D * 2;
    const uint64_t q_org = (uint64_t)((const char*)Qg - (const char*)a.qkv);
    const uint64_t do_org = (uint64_t)((const char*)dOg - (const char*)a.dout);
    constexpr int NMW = KW * BQ / NT;  // keep words staged per thread
    uint32_t rmw[NMW];
    // this (b, h)'s keep words [ntw][T] (attn_dropmask_kernel layout); an empty range without dropout
    const __amdgpu_buffer_rsrc_t mw_rs =
        kv_rsrc(reinterpret_cast<const bf16_t*>(a.thr ? a.dmask : nullptr) , a.thr ? (uint64_t)(bh + 1) * ntw * a.T * 4 : 0,
                a.thr ? (uint64_t)bh * ntw * a.T * 4 : 0);
    // Every load below is unconditional (indices clamped) and its raw value is only selected at
    // commit(): a load whose result a select right behind it needed (hipcc sank it into a branch)
    // made the wave wait vmcnt(0) just after this tile's Q / dO prefetch was issued -- a full
    // memory latency per tile in every wave.
    float rl_raw = 0.f;
    const uint32_t nodrop = a.thr ? 0u : 0xffffffffu;  // no dropout: every key kept
    auto issue = [&](int qt) {
      stq::load_buf(rq, a.qkv, q_total, q_org + (uint64_t)qt * BQ * ld * 2, oq);
      stq::load_buf(rd, a.dout, do_total, do_org + (uint64_t)qt * BQ * a.D * 2, od);
      const int t = threadIdx.x;
      // threads [0, BQ): lse, [BQ, 2 BQ): delta (the rest load a valid row and drop it)
      rl_raw = ((t & BQ) ? dlg : lseg)[min(qt * BQ + (t & (BQ - 1)), a.T - 1)];
      // keep words: word j of query row q -> sMW[j * BQ + q] (an empty descriptor without dropout)
#pragma unroll
      for (int i = 0; i < NMW; ++i) {
        const int u = t + NT * i;
        const int q = qt * BQ + (u & (BQ - 1)), j = u / BQ;
        const uint32_t off = (uint32_t)(((t0w + min(j, ntw - 1 - t0w)) * a.T + min(q, a.T - 1)) * 4);
        rmw[i] = __builtin_amdgcn_raw_buffer_load_b32(mw_rs, off, 0, 0);
      }
    };
    auto commit = [&](int qt) {
      stq::store(smem + OFF_Q, rq);
      stq::store(smem + OFF_DO, rd);
      const int t = threadIdx.x;
      const int ql = qt * BQ + (t & (BQ - 1));
      // -lse: the S init (K holds c K); delta' = delta / dscale (bwd_softmax_grad)
      const float rl = ql < a.T ? ((t & BQ) ? rl_raw * ddl : -rl_raw) : 0.f;
      if (t < 2 * BQ) reinterpret_cast<float*>(smem + OFF_L)[t] = rl;
#pragma unroll
      for (int i = 0; i < NMW; ++i) {
        const int u = t + NT * i;
        const int q = qt * BQ + (u & (BQ - 1)), j = u / BQ;
        const uint32_t w = ((q < a.T && t0w + j < ntw) ? rmw[i] : 0u) | nodrop;
        reinterpret_cast<uint32_t*>(smem + OFF_MW)[u] = w;
      }
    };
    issue(qt0);
    commit(qt0);
    __syncthreads();

    for (int qt = qt0; qt < nqt; ++qt) {
      const char* sQ = smem + OFF_Q;
      const char* sdO = smem + OFF_DO;
      int lane = threadIdx.x & 63;
      asm volatile("" : "+v"(lane));  // recomputed per tile: keeps the offsets below out of the loop state
      const int h32 = lane >> 5, l32 = lane & 31;
      const bool more = qt + 1 < nqt;
      const int qbase = qt * BQ;
      // dQ bookkeeping of this tile: first key block stores, later ones read-add-store, the last
      // one to reach the tile writes bf16
      const int last_kb = min(nkb - 1, (qbase + BQ - 1) / KB);
      const bool first = part || kb == 0, last = !part && kb == last_kb;
      if (more) issue(qt + 1);
      // previous key blocks' dQ sums of this wave's tiles: LDS-DMA'd now (no registers held),
      // added after the dQ MFMAs (a load in the store loop exposed a memory latency per tile)
      float* pvs = reinterpret_cast<float*>(smem + OFF_PV) + (my_split == 0 ? w : 0) * NTW * 16 * 64;
      if (PERSIST && !first && my_split == 0) {
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
          const int tt = tt0 + i * TSTEP;
          if (tt < TILES) {
            const int qs = tt / NO, n = tt % NO;
            const int q0 = qbase + qs * 32 + 4 * h32;
            const int d = min(n * 32 + l32, a.hd - 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int q = min(q0 + (r & 3) + 8 * (r >> 2), a.T - 1);  // rows past T: unused
              __builtin_amdgcn_global_load_lds(a.dq + ((long)b * a.T + q) * a.D + hh * a.hd + d,
                                               (__attribute__((address_space(3))) void*)(pvs + (i * 16 + r) * 64),
                                               4, 0, 0);
            }
          }
        }
      }
      char* myds = sdS + w * 32 * ROWB;
      int ro[NKS], rk_[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        ro[ks] = (ks >> 2) * HQ + lds_off(l32, (2 * ks + h32) & 7);
        rk_[ks] = (ks >> 2) * HK + 32 * w * ROWB + lds_off(l32, (2 * ks + h32) & 7);
      }
      const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int ta0 = tr_off(4 * h32 + trq, trc), tb0 = tr_off(8 + 4 * h32 + trq, trc);
      const int ta1 = tr_off(4 * h32 + trq, 32 + trc), tb1 = tr_off(8 + 4 * h32 + trq, 32 + trc);
#pragma unroll
      for (int qs = 0; qs < NQS; ++qs) {
        const int qsub0 = qbase + qs * 32;
        char* mydsh = myds + (qs >> 1) * KB * ROWB;  // dS^T half of this subtile's 64 queries
        if (qsub0 + 31 < wave_kmin || wave_kmin >= a.T) {  // every query precedes every key: dS = 0
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int qc = (qs & 1) * 32 + 8 * g + 4 * h32;
            *reinterpret_cast<uint2*>(mydsh + lds_off(l32, qc >> 3) + (qc & 7) * 2) = make_uint2(0, 0);
          }
          continue;
        }
        float dl[16];
        uint32_t mwr[16];
        f32x16 sacc, dp = {0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // row constants of this lane's 16 rows, 4 per ds_read_b128
          const int q4 = qs * 32 + 8 * g + 4 * h32;
          const float4 x = *reinterpret_cast<const float4*>(sL + q4);
          const float4 y = *reinterpret_cast<const float4*>(sL + BQ + q4);
          sacc[4 * g] = x.x; sacc[4 * g + 1] = x.y; sacc[4 * g + 2] = x.z; sacc[4 * g + 3] = x.w;
          dl[4 * g] = y.x; dl[4 * g + 1] = y.y; dl[4 * g + 2] = y.z; dl[4 * g + 3] = y.w;
          const uint4 m4 = *reinterpret_cast<const uint4*>(sMW + mw_col * BQ + q4);
          mwr[4 * g] = m4.x; mwr[4 * g + 1] = m4.y; mwr[4 * g + 2] = m4.z; mwr[4 * g + 3] = m4.w;
        }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {  // S' = Q (cK)^T - lse ; dP~ = dO V^T
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sQ + qs * 32 * ROWB, ro[ks]),
                                                         lds_row_at(sK, rk_[ks]), sacc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_row_at(sdO + qs * 32 * ROWB, ro[ks]), vf[ks], dp,
                                                       0, 0, 0);
        }
        // wave-uniform: only diagonal / past-T tiles pay for the causal mask
        if (wave_kmin + 31 > qsub0 || qsub0 + 31 >= a.T)
          bwd_softmax_grad<true>(sacc, dp, dl, mwr, a.T, mykey, mw_bit, qsub0 + 4 * h32);
        else
          bwd_softmax_grad<false>(sacc, dp, dl, mwr, a.T, mykey, mw_bit, qsub0 + 4 * h32);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pf = pack_frag(sacc, st);
          const bf16x8 dsf = pack_frag(dp, st);
          const int rb = (qs * 32 + 16 * st) * ROWB;  // 16-row aligned: an immediate
#pragma unroll
          for (int n = 0; n < NO; ++n) {
            const int hb = (n >> 1) * HQ + rb;
            const bool odd = n & 1;
            dv[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                odd ? lds_tr_at(sdO + hb, ta1, tb1) : lds_tr_at(sdO + hb, ta0, tb0), pf, dv[n], 0, 0, 0);
            dk[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                odd ? lds_tr_at(sQ + hb, ta1, tb1) : lds_tr_at(sQ + hb, ta0, tb0), dsf, dk[n], 0, 0, 0);
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // dS^T image row = key, 4 consecutive q per 8-byte write
          const int qc = (qs & 1) * 32 + 8 * g + 4 * h32;
          *reinterpret_cast<uint2*>(mydsh + lds_off(l32, qc >> 3) + (qc & 7) * 2) =
              make_uint2(pack2(dp[4 * g], dp[4 * g + 1]), pack2(dp[4 * g + 2], dp[4 * g + 3]));
        }
      }
      __syncthreads();  // dS of all KB keys in LDS
      // the next tile's Q / dO / row constants / keep words into LDS now: the dQ products below
      // read only dS^T and K, and committing before the dQ stores keeps the wait for this tile's
      // loads (and any spill reload there) from draining those stores
      if (more) commit(qt + 1);
      // dQ[BQ q][hd] = dS[BQ q][KB keys] (c K)[KB keys][hd]
#pragma unroll
      for (int i = 0; i < NTW; ++i) {
        const int tt = tt0 + i * TSTEP;
        if (tt >= TILES) break;
        const int qs = tt / NO, n = tt % NO;
        const int klo = my_split * KSPAN;
        const bool act = n * 32 < a.hd && qbase + qs * 32 + 31 >= kb0 + klo && kb0 + klo < a.T;
        f32x16 dq = {0};
        if (act) {
          // rows klo + 16 kk + 8 h32 + q (+4): the 16 kk part is an immediate
          const int qcol = (qs & 1) * 32 + trc;
          const int da = tr_off(8 * h32 + trq, qcol), db = tr_off(8 * h32 + 4 + trq, qcol);
          const int ka = tr_off(8 * h32 + trq, (n & 1) * 32 + trc), kb4 = tr_off(8 * h32 + 4 + trq, (n & 1) * 32 + trc);
          const char* sdSh = sdS + (qs >> 1) * KB * ROWB + klo * ROWB;
          const char* sKh = sK + (n >> 1) * HK + klo * ROWB;
#pragma unroll
          for (int kk = 0; kk < KSPAN / 16; ++kk)
            dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_at(sdSh + kk * 16 * ROWB, da, db),
                                                         lds_tr_at(sKh + kk * 16 * ROWB, ka, kb4), dq, 0, 0, 0);
        }
        if constexpr (KSPLIT > 1) {  // key splits 1.. hand their partial tile to split 0 via LDS
          float* part = reinterpret_cast<float*>(smem + OFF_P);
          if (my_split > 0) {
            // [split][tile][g][lane] f32x4: consecutive lanes 16 B apart (conflict-free b128)
            float* pp = part + ((my_split - 1) * TILES + tt) * 4 * 64 * 4 + lane * 4;
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *reinterpret_cast<f32x4*>(pp + g * 64 * 4) = f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
          }
          __syncthreads();
          if (my_split == 0) {
#pragma unroll
            for (int sp = 1; sp < KSPLIT; ++sp) {
              const float* pp = part + ((sp - 1) * TILES + tt) * 4 * 64 * 4 + lane * 4;
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(pp + g * 64 * 4);
                dq[4 * g] += x[0]; dq[4 * g + 1] += x[1]; dq[4 * g + 2] += x[2]; dq[4 * g + 3] += x[3];
              }
            }
          }
        }
        const int d = n * 32 + l32;
        if (part && my_split == 0 && d < a.hd && qbase + qs * 32 + 31 >= kb0) {
          // key-block partial: buffer stores through one descriptor per query tile whose extent
          // ends at row T of this sequence (rows past it are dropped: no per-row branches), row
          // offsets in SGPRs (no 64-bit address math per store)
          const uint64_t org = ((uint64_t)kb * a.dq_part + ((uint64_t)b * a.T + qbase) * a.D + (uint64_t)hh * a.hd) * 4;
          const uint64_t end = ((uint64_t)kb * a.dq_part + ((uint64_t)b + 1) * a.T * a.D) * 4;
          const __amdgpu_buffer_rsrc_t rs = kv_rsrc(reinterpret_cast<const bf16_t*>(a.dq), end, org);
          const int voff = ((qs * 32 + 4 * h32) * a.D + d) * 4;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dq[r]), rs, voff, ((r & 3) + 8 * (r >> 2)) * a.D * 4, 0);
        } else if (my_split == 0 && d < a.hd && qbase + qs * 32 + 31 >= kb0) {
          if (PERSIST && !first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
          // row q0 + (r & 3) + 8 (r >> 2): one 64-bit base per lane, then uniform row strides
          const int q0 = qbase + qs * 32 + 4 * h32;
          const long roff = ((long)b * a.T + q0) * a.D + hh * a.hd + d;
          float* dqb = a.dq + (part ? kb * a.dq_part : 0) + roff;
          bf16_t* outq = a.dqkv + ((long)b * a.T + q0) * ld + hh * a.hd + d;
          auto put = [&](int r) {
            const int dr = (r & 3) + 8 * (r >> 2);
            const float v = (!PERSIST || first) ? dq[r] : dq[r] + pvs[(i * 16 + r) * 64 + lane];
            if (last)
              outq[(long)dr * ld] = f2bf(v * dq_scale);
            else
              dqb[(long)dr * a.D] = v;
          };
          if (qbase + BQ <= a.T) {  // whole tile inside the sequence: no per-row checks
#pragma unroll
            for (int r = 0; r < 16; ++r) put(r);
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (q0 + (r & 3) + 8 * (r >> 2) < a.T) put(r);
          }
        }
      }
      __syncthreads();
    }

    // dK (scaled), dV (dropout keep scale folded) -> dqkv K / V slots; lane = key,
    // d = n*32 + 8*(r>>2) + 4*h32 + (r&3)
    const int lane = threadIdx.x & 63, h32 = lane >> 5;
    if (mykey < a.T) {
      const float sc = a.scale_log2 * 0.6931471805599453f * a.dscale;  // dscale / sqrt(hd)
      const float vs = a.thr ? a.dscale : 1.f;
      bf16_t* krow = a.dqkv + ((long)b * a.T + mykey) * ld + a.D + hh * a.hd;
      bf16_t* vrow = krow + a.D;
#pragma unroll
      for (int n = 0; n < NO; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = n * 32 + 8 * g + 4 * h32;
          if (d < a.hd) {
            *reinterpret_cast<uint2*>(krow + d) = make_uint2(pack2(dk[n][4 * g] * sc, dk[n][4 * g + 1] * sc),
                                                             pack2(dk[n][4 * g + 2] * sc, dk[n][4 * g + 3] * sc));
            *reinterpret_cast<uint2*>(vrow + d) = make_uint2(pack2(dv[n][4 * g] * vs, dv[n][4 * g + 1] * vs),
                                                             pack2(dv[n][4 * g + 2] * vs, dv[n][4 * g + 3] * vs));
          }
        }
    }
    if constexpr (!PERSIST) {
      if (a.dbias) {
        // qkv bias gradient, K and V columns: this block's keys summed in registers (lanes), the
        // KW waves through LDS (free: every read of the last tile is behind its final barrier),
        // then one fp32 atomic per column -- the separate 300 MB column-sum pass over dqkv is gone
        constexpr int NV = 32 * NO;  // this lane's dK then dV values
        float v[NV];
        const bool kv = mykey < a.T;
        const float sc = a.scale_log2 * 0.6931471805599453f * a.dscale;
        const float vs = a.thr ? a.dscale : 1.f;
#pragma unroll
        for (int n = 0; n < NO; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[n * 16 + r] = kv ? dk[n][r] * sc : 0.f;
            v[16 * NO + n * 16 + r] = kv ? dv[n][r] * vs : 0.f;
          }
        tr_reduce32<16, NV, NV>(v, lane);
        float* red = reinterpret_cast<float*>(smem);  // [KW][NO][64]
#pragma unroll
        for (int j = 0; j < NO; ++j) red[(w * NO + j) * 64 + lane] = v[j];
        __syncthreads();
        for (int t = threadIdx.x; t < 64 * NO; t += NT) {
          const int ln = t & 63, j = t >> 6;
          float s = 0.f;
#pragma unroll
          for (int ww = 0; ww < KW; ++ww) s += red[(ww * NO + j) * 64 + ln];
          const int idx = NO * (ln & 31) + j;  // value index (tr_reduce32)
          const int tk = idx / (16 * NO), n = (idx % (16 * NO)) / 16, r = idx % 16;
          const int d = n * 32 + 8 * (r >> 2) + 4 * (ln >> 5) + (r & 3);
          if (d < a.hd) atomicAdd(a.dbias + (1 + tk) * a.D + hh * a.hd + d, s);
        }
      }
    }
  }
}

// S / dP~ MFMAs of attn_bwd64_kernel, pinned to VGPR accumulators (the softmax gradient reads them
// with VALU; hipcc's own choice at this register budget was the accumulator file plus a
// v_accvgpr_read per element).  hipcc neither pads nor orders inside these statements, so the
// hazards are handled here: the first MFMA of a chain waits 2 states for a VALU-written C, and the
// chain's result is first read by VALU a whole stage later (attn_bwd64_kernel's pinned schedule
// puts 8 dV / dK MFMAs between the chain's end and that read; tests/test_isa_hazards.py checks).
MG_DEVICE void mfma_v_init(f32x16& acc, const bf16x8& a, const bf16x8& b, const f32x16& c) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=v"(acc) : "v"(a), "a"(b), "v"(c));
}
MG_DEVICE void mfma_v_zero(f32x16& acc, const bf16x8& a, const bf16x8& b) {  // C = 0
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(acc) : "v"(a), "a"(b));
}
MG_DEVICE void mfma_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}
// An MFMA reads its C operand late: a register it takes as C (the chain's initial S) must not be
// rewritten for ~11 wait states -- keep_live extends the value's live range to a later point.
MG_DEVICE void keep_live(const f32x16& v) { asm volatile("" ::"v"(v)); }

#ifdef MG_BWD64_STAMPS
// Diagnostic build only (-DMG_BWD64_STAMPS): s_memtime per wave at 8 points of each tile of the
// first 64 workgroups (bench/dev/bwd64_stamps.py reads them back).  Nothing else reads this buffer.
__device__ unsigned long long g_bwd64_stamps[64 * 4 * 8 * 8];
// per wave and for its first two work items: s_memtime and s_memrealtime (100 MHz) at the item's
// start (kernel start / the previous item's end), before the tile loops, after them, and at its end
__device__ unsigned long long g_bwd64_pe[64 * 4 * 16];
#define BWD64_PE(pt)                                                                               \
  do {                                                                                             \
    if (bwd64_it < 2 && blockIdx.x < 64 && (threadIdx.x & 63) == 0) {                              \
      g_bwd64_pe[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + 8 * bwd64_it + 2 * (pt)] = __builtin_amdgcn_s_memtime(); \
      g_bwd64_pe[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + 8 * bwd64_it + 2 * (pt) + 1] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                              \
  } while (0)
#define BWD64_STAMP(tile, pt)                                                                      \
  do {                                                                                             \
    if (bwd64_it == 0 && blockIdx.x < 64 && (tile) < 8 && (threadIdx.x & 63) == 0)                 \
      g_bwd64_stamps[((blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (tile)) * 8 + (pt)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define BWD64_PE(pt) \
  do {               \
  } while (0)
#define BWD64_STAMP(tile, pt) \
  do {                        \
  } while (0)
#endif

// One LDS-DMA dword per lane (64 consecutive dwords at LDS byte address lds, a wave-uniform value)
// from a buffer: inline asm so that hipcc neither counts it (it would put vmcnt(0) in front of every
// later LDS read it cannot tell apart from the DMA's writes) nor keeps a register for it.  M0 is
// saved and restored inside the statement; the completion is waited for by the caller.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// kv_rsrc's descriptor as four scalar words (what an asm operand can take)
MG_DEVICE u32x4_t kv_rsrc_words(const void* base, uint64_t total, uint64_t off) {
  const uint64_t p = reinterpret_cast<uint64_t>(base) + off;
  const uint64_t left = off < total ? total - off : 0;
  u32x4_t d;
  d[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
  d[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32) & 0xffffu);
  d[2] = __builtin_amdgcn_readfirstlane((uint32_t)(left < 0xffffffffull ? left : 0xffffffffull));
  d[3] = 0x00020000u;
  return d;
}
MG_DEVICE void dma_dwordx4(const u32x4_t& rs, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds), "s"(soff)
      : "memory");
}
MG_DEVICE void dma_dword(const u32x4_t& rs, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds), "s"(soff)
      : "memory");
}

// =================================================================== backward, head dim 64
// Key-block backward for hd = 64 (every GPT-2 size), one wave per SIMD.  Same grid, LDS images,
// dQ partials and finalize as attn_bwd_kernel<4, 8, false>, and the same arithmetic in the same
// order (its outputs are bitwise those of that kernel), but organised for instruction-level
// parallelism inside the wave instead of a second wave per SIMD:
//  * 4 waves x 64 keys: wave w owns key groups 2w and 2w + 1 (32 keys each, key on the lane).  A
//    "unit" is one 32-query subtile x one key group: S and dP~ (8 MFMAs), the softmax gradient
//    (VALU), dV^T / dK^T (8 MFMAs), its dS^T into LDS.  The two groups of a subtile share its Q / dO
//    row fragments (S / dP~ A operands) and its transposed dO^T / Q^T fragments (dV / dK A operands),
//    so each is read from LDS once per two units; the groups' K and V rows stay in registers.
//  * software pipeline over the 8 units of a 128-query tile: unit u+1's S / dP~ MFMAs are issued
//    beside unit u's softmax-gradient VALU (two accumulator pairs), so the matrix pipe works while
//    the vector pipe does; the whole tile is one basic block (no per-unit branches).
//  * the causal mask is folded into the S accumulator's initial value (-lse, or -inf where the key
//    follows the query): exp2 gives exactly 0 there, so masked, skipped and diagonal units all run
//    the same straight-line code; only diagonal tiles (some key of the block after some query of
//    the tile) pay the per-element select, in a second instance of the tile body.  Rows past T
//    carry -inf from staging.
//  * every LDS address is a per-lane base computed once per kernel plus an immediate.
// Register budget: dK^T / dV^T of 2 groups (128), K / V fragments (64), two S / dP~ pairs (64), the
// next tile's staged Q / dO (32), row constants of two subtiles (64), operand fragments.
__global__ __launch_bounds__(256, 1) void attn_bwd64_kernel(const AttnArgs a) {
  [[maybe_unused]] int bwd64_it = 0;  // stamps (diagnostic build): the work item's ordinal
  BWD64_PE(0);
  constexpr int BQ = 128, KB = 256, NT = 256, NKS = 4, NO = 2, KW = 8;
  constexpr int HQ = BQ * ROWB;
  constexpr int OFF_Q = 0, OFF_DO = HQ, OFF_K = 2 * HQ, OFF_DS = OFF_K + KB * ROWB;
  constexpr int OFF_L = OFF_DS + 2 * KB * ROWB, OFF_MW = OFF_L + 2 * BQ * 4;
  constexpr int MWB = KW * BQ * 4;  // one tile's keep words; two buffers (tile parity)
  constexpr int OFF_DO2 = OFF_MW + 2 * MWB;  // dO image of odd tiles (even tiles: OFF_DO)
  constexpr int OFF_ITEM = OFF_DO2 + HQ;     // the next work item (one int)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h32 = lane >> 5, l32 = lane & 31;
  const int BH = a.B * a.H;
  const long ld = 3L * a.D;
  const int ntw = 2 * ((a.T + 63) / 64);
  const int nqt = (a.T + BQ - 1) / BQ;
  const int n_items = BH * ((a.T + KB - 1) / KB);

  char* const sQ = smem + OFF_Q;
  char* const sK = smem + OFF_K;
  char* const sdS = smem + OFF_DS;
  int* const sItem = reinterpret_cast<int*>(smem + OFF_ITEM);
  using stk = Stager<KB, 1, NT>;

  // ---- work items: (key block, b, h) = (item / BH, item % BH), heaviest key blocks first.  Each
  // workgroup takes blockIdx.x, then the next free item from the counter (zeroed by
  // attn_bwd_pre_kernel): a workgroup that starts late (CUs held by a concurrent kernel) takes
  // fewer.  The next item is known one item ahead, so its K / V / first-tile loads are issued
  // under the current item's last tile and epilogue instead of after them.
  int item = blockIdx.x;
  int bh, kb, b, hh, kb0, qt0;
  int mykey[2];
  auto setup = [&](int it) {
    bh = it % BH;
    kb = it / BH;
    b = bh / a.H;
    hh = bh % a.H;
    kb0 = kb * KB;
    qt0 = kb0 / BQ;
#pragma unroll
    for (int g = 0; g < 2; ++g) mykey[g] = kb0 + 64 * w + 32 * g + l32;
  };
  setup(item);

  // K and V rows of an item, raw, by LDS-DMA into the dS^T image (K at OFF_DS, V 32 KiB on):
  // 8 rows x 128 B per instruction, 8 per wave each; rows past T read 0 (descriptor extent).  No
  // registers held while they fly (the next item's are issued before the current epilogue)
  auto dma_kv = [&](int ib, int ihh, int ikb0) {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    const int ln = t & 63;
    const uint32_t v0 = (uint32_t)((ln >> 3) * ld * 2 + (ln & 7) * 16);
    const uint64_t org = (((uint64_t)ib * a.T + ikb0) * ld + a.D + ihh * 64) * 2;
    const uint64_t ext = (uint64_t)(a.T - ikb0 - 1) * ld * 2 + 128;
    const u32x4_t rk_ = kv_rsrc_words(a.qkv, org + ext, org), rv_ = kv_rsrc_words(a.qkv, org + ext + a.D * 2, org + a.D * 2);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + OFF_DS);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pc = 8 * wv + i;  // rows 8 pc ..: in voffset, the part the range check sees
      const uint32_t v = v0 + (uint32_t)(8 * pc * ld * 2);
      dma_dwordx4(rk_, v, 0, lb + pc * 1024);
      dma_dwordx4(rv_, v, 0, lb + KB * ROWB + pc * 1024);
    }
  };
  bf16x8 vf[2][NKS];  // this wave's V rows (dP~'s B operand), group g = keys 64 w + 32 g + lane
  // after dma_kv landed (vmcnt(0) + barrier): K <- c K into its LDS image (dQ's B operand; the K
  // fragments of the chains come from it), this wave's V fragments into registers
  auto convert_kv = [&]() {
    // addresses from an opaque thread id: hoisted out of the item loop they were spilled, and the
    // reload's vmcnt(0) made the item transition wait for the epilogue's stores after all
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
    uint4 rk[stk::N];
#pragma unroll
    for (int i = 0; i < stk::N; ++i) {
      const int idx = tt + NT * i, rem = idx % (KB * 8);
      rk[i] = *reinterpret_cast<const uint4*>(sdS + (rem >> 3) * ROWB + (rem & 7) * 16);
      float f[8];
      unpack8(rk[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= a.scale_log2;
      rk[i] = pack8(f);
    }
#pragma unroll
    for (int c = 0; c < stk::N; ++c) {  // stk::store with the opaque thread id
      const int idx = tt + NT * c, rem = idx % (KB * 8);
      *reinterpret_cast<uint4*>(sK + (idx / (KB * 8)) * KB * ROWB + lds_off(rem >> 3, rem & 7)) = rk[c];
    }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        vf[g][ks] = *reinterpret_cast<const bf16x8*>(sdS + KB * ROWB + ((tt >> 6) * 64 + 32 * g + (tt & 31)) * ROWB +
                                                     ks * 32 + 16 * ((tt >> 5) & 1));
  };
  dma_kv(b, hh, kb0);
  // dropout: both groups read the same keep word of a row (the 64-key tile of keys 64 w..), the
  // second group's bit 8 above the first's (attn_dropmask_kernel layout)
  const int mw_col = 2 * w + ((l32 >> 2) & 1);
  const int mw_bit0 = drop_bit((l32 & 3) | (((l32 >> 3) & 3) << 2));

  // ---- per-lane LDS offsets, computed once (every access below adds an immediate)
  int ro[NKS];  // row-fragment reads (Q, dO, K): row l32, chunk 2 ks + h32
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) ro[ks] = lds_off(l32, (2 * ks + h32) & 7);
  // transposed reads (dO^T / Q^T): rows 4 h32 + trq (ta) and 8 more (tb), columns trc (+ 32 n).
  // With tr_off's swizzle, column + 32 flips bit 6 of the offset and row + 8 flips it again and
  // adds 1024: ta[0] = ta0, ta[1] = ta0 ^ 64, tb[0] = ta[1] + 1024, tb[1] = ta0 + 1024 (two
  // registers; the 1024 lands in the instruction's offset field)
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int ta0 = tr_off(4 * h32 + trq, trc), ta0x = ta0 ^ 64;
  // dS^T image writes: key row 64 w + l32 (+ 32 g), query chunk j at wbase + ((16 j) ^ wsw) (two
  // registers and one v_xad per write instead of 8 offsets held across the tile loop)
  const int wbase = 64 * w * ROWB + l32 * ROWB + 8 * h32, wsw = swz(l32) << 4;
  const int rowL = OFF_L + 16 * h32;                     // + 4 (32 qs + 8 g')
  const int rowMW0 = OFF_MW + 4 * (mw_col * BQ + 4 * h32);  // + 4 (32 qs + 8 g'), + MWB on odd tiles

  f32x16 dk[2][NO], dv[2][NO];
  auto zero_acc = [&]() {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int n = 0; n < NO; ++n) {
        dk[g][n] = f32x16{0};
        dv[g][n] = f32x16{0};
      }
  };
  zero_acc();

  // ---- next-tile staging, in registers (the LDS has no room for a second Q / dO image).  Every
  // load goes through a descriptor with ONE per-lane base offset; the chunk and tile parts ride in
  // the scalar offset.  (Per-chunk offset registers were spilled, and each reload's vmcnt(0) put
  // the tile's loads behind one another: 13k cycles per tile.)
  // (per-lane offsets recomputed inside issue / commit from an opaque thread id: kept live across
  // the tile loop they were spilled too)
  uint4 rq[4];  // Q, chunk c: tile row t / 8 + 32 c, 16-byte chunk t % 8 (dO goes by LDS-DMA)
  const uint64_t q_total = (uint64_t)a.B * a.T * ld * 2, do_total = (uint64_t)a.B * a.T * a.D * 2;
  float rl_raw = 0.f;
  // tile qt of the current item (bh, kb) into the LDS buffers of parity par.  Keep words: word row
  // t0w + j (j = t / 128 + 2 i), query row q of the tile, DMA'd to LDS as they are (a word of a row
  // past T or of keys past T meets p = 0 in the softmax -- the -inf rows and the causal mask -- so
  // its value never matters; reads past this (b, h)'s words return 0 by the descriptor extent).
  // Without dropout the LDS words are set to all-ones once.  Row constants: waves 0-1 load lse,
  // waves 2-3 delta (threads [0, BQ) / [BQ, 2 BQ)); rows past T read 0 (descriptor extent) and
  // are replaced at commit.
  // descriptors of the item whose tiles issue() stages, built once per item (set_issue_item), not
  // per tile: the 64-bit origin arithmetic of four descriptors ran on the CU's one scalar unit for
  // all four waves at every tile.  Every row-dependent offset rides in voffset -- the part the
  // hardware range-checks -- so rows past the end of a tensor read 0.
  u32x4_t dmw = {0u, 0u, 0u, 0u}, ddo;
  __amdgpu_buffer_rsrc_t dqr, dlr;
  int dt0w = 0;
  auto set_issue_item = [&](int ib, int ihh, int ibh, int ikb0) {
    dt0w = (ikb0 / 64) * 2;
    if (a.thr) dmw = kv_rsrc_words(a.dmask, (uint64_t)(ibh + 1) * ntw * a.T * 4, (uint64_t)ibh * ntw * a.T * 4);
    ddo = kv_rsrc_words(a.dout, do_total, ((uint64_t)ib * a.T * a.D + (uint64_t)ihh * 64) * 2);
    dqr = kv_rsrc(a.qkv, q_total, ((uint64_t)ib * a.T * ld + (uint64_t)ihh * 64) * 2);
    dlr = kv_rsrc(reinterpret_cast<const bf16_t*>((w >= 2 ? a.delta : a.lse) + (long)ibh * a.T), (uint64_t)a.T * 4, 0);
  };
  auto issue = [&](int qt, int par) {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    if (a.thr) {  // keep words straight into LDS buffer par, issued first (see commit)
      const uint32_t vmw = (uint32_t)(((t >> 7) * a.T + (t & (BQ - 1)) + dt0w * a.T + qt * BQ) * 4);
      const uint32_t lb = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + OFF_MW + par * MWB + 64 * 4 * (threadIdx.x >> 6)));
#pragma unroll
      for (int i = 0; i < 4; ++i) dma_dword(dmw, vmw + (uint32_t)(2 * i * a.T * 4), 0, lb + NT * 4 * i);
    }
    {  // dO straight into its LDS image for tile qt (buffer par): 16 pieces of 8 rows x 128 B,
       // 4 per wave; lane -> (row 8 p + lane / 8, stored chunk lane % 8), the swizzle applied on
       // the source side (logical chunk = stored ^ swz(row); swz's bit 2 follows the piece parity)
      const int ln = t & 63, r8 = ln >> 3;
      const uint32_t vt = (uint32_t)((qt * BQ + r8) * a.D * 2);
      const uint32_t v0 = vt + (uint32_t)((((ln & 7) ^ swz(r8)) << 4));
      const uint32_t v1 = vt + (uint32_t)((((ln & 7) ^ swz(r8 + 8)) << 4));
      const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t lb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + (par ? OFF_DO2 : OFF_DO));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pc = 4 * wv + i;  // piece: rows 8 pc ..
        dma_dwordx4(ddo, ((i & 1) ? v1 : v0) + (uint32_t)(8 * pc * a.D * 2), 0, lb + pc * 1024);
      }
    }
    const uint32_t vq = (uint32_t)(((t >> 3) + qt * BQ) * ld * 2 + (t & 7) * 16);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      rq[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dqr, vq + (uint32_t)(c * 32 * ld * 2), 0, 0));
    rl_raw = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dlr, (uint32_t)(((t & (BQ - 1)) + qt * BQ) * 4), 0, 0));
  };
  auto commit = [&](int qt) {
    // this wave's DMA'd dO rows and keep words (issued before every load waited for here) have
    // landed; the barrier after the tile publishes them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    const int wq = lds_off(t >> 3, t & 7);  // + 32 c rows: an immediate (swizzle period 16 rows)
#pragma unroll
    for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(sQ + wq + c * 32 * ROWB) = rq[c];
    const int ql = qt * BQ + (t & (BQ - 1));
    // S init = -lse (K holds c K), -inf on rows past T: exp2 gives 0 there; delta' = delta / dscale
    // (1 / dscale computed here: held across the tile loop it was spilled; times the reciprocal,
    // not a division, as attn_bwd_kernel does)
    const float rl = (t & BQ) ? (ql < a.T ? rl_raw * (1.f / a.dscale) : 0.f) : (ql < a.T ? -rl_raw : -INFINITY);
    reinterpret_cast<float*>(smem + OFF_L)[t] = rl;
  };
  if (!a.thr) {  // no dropout: every key kept (both buffers)
#pragma unroll
    for (int i = 0; i < 8; ++i) reinterpret_cast<uint32_t*>(smem + OFF_MW)[threadIdx.x + NT * i] = 0xffffffffu;
  }
  int par = 0;  // LDS buffer parity of the current tile's dO image and keep words
  set_issue_item(b, hh, bh, kb0);
  issue(qt0, par);
  if (threadIdx.x == 0) *sItem = atomicAdd(a.work, 1) + (int)gridDim.x;  // the item after this one
  commit(qt0);  // its vmcnt(0) covers dma_kv
  __syncthreads();
  convert_kv();
  __syncthreads();

  int nxt = 0, nbh = 0, nb = 0, nhh = 0, nkb0 = 0;  // the next item (valid if has_next)
  int nn_raw = 0;  // thread 0: the counter value of the item after the next one
  bool has_next = false;
  // one 128-query tile; DIAG: some key of the block follows some query of the tile.  The diagonal
  // tiles (the first two of the block) and the rest run in two loops, each with ONE instance of the
  // tile body: one body per loop keeps the register assignment of the loop-carried accumulators
  // fixed (two bodies in one loop made hipcc shuffle them between files at every tile)
  auto run_tile = [&](int qt, auto diag_tag) {
    constexpr bool DIAG = decltype(diag_tag)::value;
    const bool more = qt + 1 < nqt;
    const int qbase = qt * BQ;
    const int rowMW = rowMW0 + par * MWB;
    const char* const sdO = smem + (par ? OFF_DO2 : OFF_DO);  // this tile's dO image
    BWD64_STAMP(qt - qt0, 0);
    const int qn = more ? qt + 1 : nkb0 / BQ;  // the next tile: this item's, or the next item's first
    if (!more && has_next) set_issue_item(nb, nhh, nbh, nkb0);
    if (more || has_next) issue(qn, par ^ 1);
    BWD64_STAMP(qt - qt0, 1);
    // one 128-query tile: 8 units (subtile qs = u / 2, key group g = u % 2) in a three-deep
    // software pipeline.  Stage u (0..8) is 16 slots, each ONE MFMA plus one element of unit u's
    // softmax gradient (exp, keep select, 2 FMAs: about one MFMA gap of vector issue):
    //   even slot 2k: MFMA k of unit u+1's S / dP~ chain
    //   odd slot 2m+1: MFMA m of unit u-1's dV^T / dK^T (its P / dS packed in stage u-1)
    // plus, each where the registers it overwrites have been read for the last time and a few slots
    // ahead of its first use: bf16 packs and dS^T writes of unit u, the K-fragment ring, the next
    // subtile's Q / dO / Q^T / dO^T fragments and row constants, the next chain's initial S.  A
    // sched_barrier after every slot pins this order (hipcc left alone issued each chain as one
    // burst and the vector work after it).  The chain's results are first read a stage later.
    auto tile = [&](auto) {
      bf16x8 qf[NKS], df[NKS];           // Q / dO row fragments of the chain's subtile
      bf16x8 kfb[2];                     // K-fragment ring of the chain (S's B operand)
      bf16x8 atr[NO][2], qtr[NO][2];     // dO^T / Q^T fragments of the dV / dK unit's subtile
      bf16x8 pf[2], dsf[2];              // that unit's bf16 P / dS, by 16-query step
      f32x16 sacc[2], dpa[2], sinit;     // S / dP~ of units u (by u & 1); next chain's initial S
      float dl[16];                      // delta' of the softmax unit's rows
      uint32_t mwr[16];                  // their keep words
      auto kfrag = [&](int g, int ks) { return lds_row_at(sK + (64 * w + 32 * g) * ROWB, ro[ks]); };
      auto ld_qd = [&](int qs, int ks) {
        qf[ks] = lds_row_at(sQ + qs * 32 * ROWB, ro[ks]);
        df[ks] = lds_row_at(sdO + qs * 32 * ROWB, ro[ks]);
      };
      auto ld_tr = [&](int qs, int st) {
        const int rb = (qs * 32 + 16 * st) * ROWB;
#pragma unroll
        for (int n = 0; n < NO; ++n) {
          const int oa = n ? ta0x : ta0, ob = n ? ta0 : ta0x;  // tb[n] = ob + 1024
          atr[n][st] = lds_tr_at(sdO + rb, oa, ob + 1024);
          qtr[n][st] = lds_tr_at(sQ + rb, oa, ob + 1024);
        }
      };
      auto ld_rows = [&](int qs, int g4) {
        const float4 y = *reinterpret_cast<const float4*>(smem + rowL + 4 * BQ + 4 * (32 * qs + 8 * g4));
        dl[4 * g4] = y.x; dl[4 * g4 + 1] = y.y; dl[4 * g4 + 2] = y.z; dl[4 * g4 + 3] = y.w;
        const uint4 m4 = *reinterpret_cast<const uint4*>(smem + rowMW + 4 * (32 * qs + 8 * g4));
        mwr[4 * g4] = m4.x; mwr[4 * g4 + 1] = m4.y; mwr[4 * g4 + 2] = m4.z; mwr[4 * g4 + 3] = m4.w;
      };
      auto ld_init = [&](int u) {  // -lse of unit u's rows (S' = Q (cK)^T - lse)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 x = *reinterpret_cast<const float4*>(smem + rowL + 4 * (32 * (u >> 1) + 8 * g4));
          sinit[4 * g4] = x.x; sinit[4 * g4 + 1] = x.y; sinit[4 * g4 + 2] = x.z; sinit[4 * g4 + 3] = x.w;
        }
      };
      auto mask_init = [&](int u) {  // causal: -inf where key 64 w + 32 g + l32 follows the row's query
        if constexpr (DIAG) {
          const int dlt = kb0 + 64 * w + 32 * (u & 1) - qbase - 32 * (u >> 1) + l32;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (dlt > (r & 3) + 8 * (r >> 2) + 4 * h32) sinit[r] = -INFINITY;
        }
      };
      // MFMA k (0..7) of unit u's S / dP~ chain, with the K ring refill it frees
      auto chain_mfma = [&](int u, int k) {
        const int g = u & 1, ks = k >> 1;
        f32x16& sn = sacc[u & 1];
        f32x16& pn = dpa[u & 1];
        if (k & 1) {
          if (k == 1) mfma_v_zero(pn, df[0], vf[g][0]);
          else mfma_v(pn, df[ks], vf[g][ks]);
        } else {
          if (k == 0) mfma_v_init(sn, qf[0], kfb[0], sinit);
          else mfma_v(sn, qf[ks], kfb[ks & 1]);
          // the ring slot just read: this chain's fragment ks + 2, else the next chain's ks - 2
          if (ks < 2) kfb[ks & 1] = kfrag(g, ks + 2);
          else if (u + 1 < 8) kfb[ks & 1] = kfrag((u + 1) & 1, ks - 2);
        }
      };
      auto dvdk_mfma = [&](int u, int m) {  // MFMA m (0..7) of unit u's dV^T / dK^T
        const int g = u & 1, st = m >> 2, n = (m >> 1) & 1;
        if (m & 1) dk[g][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qtr[n][st], dsf[st], dk[g][n], 0, 0, 0);
        else dv[g][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(atr[n][st], pf[st], dv[g][n], 0, 0, 0);
      };
      auto pack = [&](int u, int st) {  // unit u's P / dS rows of 16-query step st, and its dS^T
        pf[st] = pack_frag(sacc[u & 1], st);
        dsf[st] = pack_frag(dpa[u & 1], st);
      };
      auto ds_write = [&](int u, int st) {  // dS^T image: row = key, 4 queries per 8-byte write
        const int qs = u >> 1, g = u & 1;
        char* dsb = sdS + (qs >> 1) * KB * ROWB + 32 * g * ROWB;
        const uint4 dw = __builtin_bit_cast(uint4, dsf[st]);
        const int j0 = (qs & 1) * 4 + 2 * st;
        *reinterpret_cast<uint2*>(dsb + wbase + ((16 * j0) ^ wsw)) = make_uint2(dw.x, dw.y);
        *reinterpret_cast<uint2*>(dsb + wbase + ((16 * (j0 + 1)) ^ wsw)) = make_uint2(dw.z, dw.w);
      };
      // ---- prologue: unit 0's chain alone, and what stage 0 needs
      kfb[0] = kfrag(0, 0);
      kfb[1] = kfrag(0, 1);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) ld_qd(0, ks);
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) ld_rows(0, g4);
      ld_init(0);
      mask_init(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) chain_mfma(0, k);
      ld_tr(0, 0);
      ld_tr(0, 1);
      ld_init(1);
      mask_init(1);
      __builtin_amdgcn_sched_barrier(0);
      float pcur = 0.f, pnext = 0.f;  // exp2 of the softmax element of this slot / the next
#pragma unroll
      for (int u = 0; u <= 8; ++u) {
        const int qs = u >> 1, g = u & 1;
        const int bit = mw_bit0 + 8 * g;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (j & 1) {
            if (u >= 1) dvdk_mfma(u - 1, j >> 1);
          } else if (u + 1 < 8) {
            chain_mfma(u + 1, j >> 1);
          }
          if (u < 8) {
            if (j == 0) pcur = fexp2(sacc[u & 1][0]);
            if (j < 15) pnext = fexp2(sacc[u & 1][j + 1]);
            bwd_softmax_one(sacc[u & 1], dpa[u & 1], dl, mwr, bit, j, pcur);
            pcur = pnext;
          }
          // ---- loads and packs placed after their registers' last reads
          if (j == 2 && u >= 1) ds_write(u - 1, 1);
          if (j == 3 && u + 1 < 8) keep_live(sinit);  // the chain's C, read late by MFMA 0
          if (j == 4 && u + 2 < 8) ld_init(u + 2);
          if (j == 8 && u < 8) pack(u, 0);  // rows 0..7 done; step-0 packs of u-1 consumed (slot 7)
          if (j == 9 && u + 2 < 8) mask_init(u + 2);
          if (j == 10 && u < 8) ds_write(u, 0);
          if (j == 15 && u < 8) pack(u, 1);  // rows 8..15 done; step-1 packs of u-1 consumed (slot 15)
          // next subtile's Q / dO rows once this stage's chain has read them (unit u+1 = (qs, 1))
          if (g == 0 && u + 1 < 8 && qs + 1 < 4 && (j & 3) == 2) ld_qd(qs + 1, j >> 2);
          // next subtile's transposed fragments once unit u-1's dV / dK read them (u starts a subtile)
          if (g == 0 && u >= 1 && u < 8 && j == 7) ld_tr(qs, 0);
          if (g == 0 && u >= 1 && u < 8 && j == 15) ld_tr(qs, 1);
          // next subtile's row constants, 4 rows at a time, once this stage's softmax read them
          if (g == 1 && u < 7 && (j & 3) == 3) ld_rows(qs + 1, j >> 2);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    tile(diag_tag);
    BWD64_STAMP(qt - qt0, 2);
    __syncthreads();  // dS^T of all 256 keys in LDS
    BWD64_STAMP(qt - qt0, 3);
    if (more || has_next) commit(qn);  // the dQ products read only dS^T and K
    // the item after the next one, fetched here (after commit's vmcnt(0)), so that its return is
    // long in by the epilogue's end, where it is published: a wait for it there would also wait
    // for every store issued before it
    if (!more && has_next && threadIdx.x == 0) nn_raw = atomicAdd(a.work, 1);
    BWD64_STAMP(qt - qt0, 4);
    // dQ[32 queries of subtile w][64] = dS (c K), over the keys that precede some query of it
    const int q0w = qbase + 32 * w;
    if (q0w + 31 >= kb0) {
      // offsets recomputed per tile from an opaque lane id: kept live across the loop they were
      // spilled (the reload's vmcnt(0) waits for the previous tile's dQ stores)
      int lo = lane;
      asm volatile("" : "+v"(lo));
      const int trq2 = (lo & 15) >> 2, trc2 = 16 * ((lo >> 4) & 1) + 4 * (lo & 3), hh32 = lo >> 5;
      const int qcol = (w & 1) * 32 + trc2;
      const int da = tr_off(8 * hh32 + trq2, qcol), db = tr_off(8 * hh32 + 4 + trq2, qcol);
      const int ka[2] = {tr_off(8 * hh32 + trq2, trc2), tr_off(8 * hh32 + trq2, 32 + trc2)};
      const int kc[2] = {tr_off(8 * hh32 + 4 + trq2, trc2), tr_off(8 * hh32 + 4 + trq2, 32 + trc2)};
      f32x16 dq[NO] = {f32x16{0}, f32x16{0}};
      const char* sdSh = sdS + (w >> 1) * KB * ROWB;
      {
        // all 16 key steps, also on diagonal tiles (the steps past the subtile's last query add
        // exact zeros; a trimmed loop of runtime length measured slower).  The fragments of step
        // kk + 4 are read while step kk's two MFMAs run (a 4-deep register ring, order pinned;
        // hipcc left alone read 4 steps, waited, ran their 8 MFMAs, then read the next 4 -- the
        // LDS latency exposed every 4 steps: 2.8k -> 1.9k cycles per tile)
        constexpr int R = 4;
        bf16x8 fa[R], fb[R][NO];
        auto ld_step = [&](int kk) {
          fa[kk % R] = lds_tr_at(sdSh + kk * 16 * ROWB, da, db);
#pragma unroll
          for (int n = 0; n < NO; ++n) fb[kk % R][n] = lds_tr_at(sK + kk * 16 * ROWB, ka[n], kc[n]);
        };
#pragma unroll
        for (int kk = 0; kk < R; ++kk) ld_step(kk);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KB / 16; ++kk) {
#pragma unroll
          for (int n = 0; n < NO; ++n)
            dq[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk % R], fb[kk % R][n], dq[n], 0, 0, 0);
          if (kk + R < KB / 16) ld_step(kk + R);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      BWD64_STAMP(qt - qt0, 5);
      // key-block partial: buffer stores through one descriptor whose extent ends at row T of
      // this sequence (rows past it are dropped), row offsets in SGPRs
      const uint64_t org = ((uint64_t)kb * a.dq_part + ((uint64_t)b * a.T + qbase) * a.D + (uint64_t)hh * 64) * 4;
      const uint64_t end = ((uint64_t)kb * a.dq_part + ((uint64_t)b + 1) * a.T * a.D) * 4;
      const __amdgpu_buffer_rsrc_t rs = kv_rsrc(reinterpret_cast<const bf16_t*>(a.dq), end, org);
#pragma unroll
      for (int n = 0; n < NO; ++n) {
        const int voff = ((32 * w + 4 * h32) * a.D + n * 32 + l32) * 4;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dq[n][r]), rs, voff, ((r & 3) + 8 * (r >> 2)) * a.D * 4, 0);
      }
    }
    BWD64_STAMP(qt - qt0, 6);
    __syncthreads();
    BWD64_STAMP(qt - qt0, 7);
    par ^= 1;
  };

  // dK (scaled), dV (dropout keep scale folded) -> dqkv K / V slots; lane = key,
  // d = n*32 + 8*(r>>2) + 4*h32 + (r&3)
  const float sc = a.scale_log2 * 0.6931471805599453f * a.dscale;  // dscale / sqrt(hd)
  const float vs = a.thr ? a.dscale : 1.f;
  // 16-byte stores (T21): the lanes l32 and l32 + 32 hold interleaved 4-column pieces of one key
  // row; one v_permlane32_swap per dword gives each the 8 contiguous columns of a 16-column step
  // (lanes < 32: columns 16 k .. + 7, the others 16 k + 8 .. + 15): half the store instructions
  // of the row-per-lane 8-byte form, which was store-issue bound
  // Buffer stores through a descriptor whose extent ends with row T - 1: every lane stores (rows
  // past T are dropped by the range check), no per-lane branch.
  auto store_row = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t voff, const f32x16 (&acc)[NO], float scale) {
#pragma unroll
    for (int n = 0; n < NO; ++n)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const f32x16& c = acc[n];
        const uint32_t x0 = pack2(c[8 * k] * scale, c[8 * k + 1] * scale), x1 = pack2(c[8 * k + 2] * scale, c[8 * k + 3] * scale);
        const uint32_t y0 = pack2(c[8 * k + 4] * scale, c[8 * k + 5] * scale), y1 = pack2(c[8 * k + 6] * scale, c[8 * k + 7] * scale);
        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{s0[0], s1[0], s0[1], s1[1]}, rs,
                                               voff + (uint32_t)((n * 32 + 16 * k) * 2), 0, 0);
      }
  };
  for (;;) {
  nxt = __builtin_amdgcn_readfirstlane(*sItem);  // published by the barrier that ended the prologue
  has_next = nxt < n_items;
  nbh = nxt % BH;
  nkb0 = (nxt / BH) * KB;
  nb = nbh / a.H;
  nhh = nbh % a.H;
  const int qdiag = min(nqt, (kb0 + KB + BQ - 1) / BQ);
  BWD64_PE(1);
  for (int qt = qt0; qt < qdiag; ++qt) run_tile(qt, std::integral_constant<bool, true>{});
  for (int qt = qdiag; qt < nqt; ++qt) run_tile(qt, std::integral_constant<bool, false>{});
  BWD64_PE(2);
  // the next item's K / V (the dS^T image is free: the last tile's dQ products are behind its
  // final barrier), under this epilogue's stores
  if (has_next) dma_kv(nb, nhh, nkb0);
  {
    const uint64_t org = ((uint64_t)b * a.T + kb0) * ld * 2;  // row kb0 of this sequence
    const __amdgpu_buffer_rsrc_t rso =
        kv_rsrc(a.dqkv, org + (uint64_t)(a.T - kb0) * ld * 2, org);  // extent: through row T - 1
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const uint32_t voff = (uint32_t)(((64 * w + 32 * g + l32) * ld + a.D + hh * 64 + 8 * h32) * 2);
      store_row(rso, voff, dk[g], sc);
      store_row(rso, voff + (uint32_t)(a.D * 2), dv[g], vs);
    }
  }
  if (a.dbias) {
    // qkv bias gradient, K and V columns (as attn_bwd_kernel, key group 2 w + g in the place of
    // its wave): keys summed over the lanes, the 8 groups through LDS, one atomic per column
    constexpr int NV = 32 * NO;
    // [8 groups][NO][64] in the dO buffer the last tile used (the Q image and the other dO buffer
    // hold the next item's first tile, the dS^T image its K / V)
    float* red = reinterpret_cast<float*>(smem + (par ? OFF_DO : OFF_DO2));
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float v[NV];
      const bool kv = mykey[g] < a.T;
#pragma unroll
      for (int n = 0; n < NO; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          v[n * 16 + r] = kv ? dk[g][n][r] * sc : 0.f;
          v[16 * NO + n * 16 + r] = kv ? dv[g][n][r] * vs : 0.f;
        }
      tr_reduce32<16, NV, NV>(v, lane);
#pragma unroll
      for (int j = 0; j < NO; ++j) red[((2 * w + g) * NO + j) * 64 + lane] = v[j];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 64 * NO; t += NT) {
      const int ln = t & 63, j = t >> 6;
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < KW; ++ww) s += red[(ww * NO + j) * 64 + ln];
      const int idx = NO * (ln & 31) + j;
      const int tk = idx / (16 * NO), n = (idx % (16 * NO)) / 16, r = idx % 16;
      const int d = n * 32 + 8 * (r >> 2) + 4 * (ln >> 5) + (r & 3);
      atomicAdd(a.dbias + (1 + tk) * a.D + hh * 64 + d, s);
    }
  }
  // the item after the next one; read after the next item's prologue barrier
  if (threadIdx.x == 0 && has_next) *sItem = nn_raw + (int)gridDim.x;
  BWD64_PE(3);
  if (!has_next) break;
  ++bwd64_it;
  BWD64_PE(0);  // the next item's start (stamps): its prologue follows
  // ---- the next item's prologue: its first tile was staged by the last tile, its K / V rows
  // DMA'd under the epilogue
  item = nxt;
  setup(item);
  zero_acc();
  // K / V landed (and this item's stores drained).  Waiting for the DMA alone -- vmcnt(16), the
  // 16 dK / dV stores being younger -- took the transition from 6.3k to 4.0k cycles but measured
  // no faster per kernel (profiles/round6_attn_bwd64_transition_ab.txt), so the count-free wait stays.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  convert_kv();
  __syncthreads();
  }
}

// partial mode: dqkv Q slot = bf16(scale * sum of the dQ partials of key blocks kb <= t / KB)
__global__ __launch_bounds__(256) void attn_dq_finalize_kernel(const float* __restrict__ dq,
                                                               bf16_t* __restrict__ dqkv, int rows,
                                                               int D, int T, int KB, long part, float sc) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over rows * D/8
  const int d8 = D / 8;
  if (i >= (long)rows * d8) return;
  const int r = (int)(i / d8);  // 32-bit operands: a cheap division
  const int c = (int)(i - (long)r * d8) * 8;
  const int np = (r % T) / KB + 1;
  const float* src = dq + (long)r * D + c;
  float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
  for (int k = 0; k < np; k += 4) {  // four partials' loads in flight before the adds
    float4 y[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // partials are read once: non-temporal
      const bool ok = k + u < np;
      const float* s = src + (long)(ok ? k + u : k) * part;
      const uint4 a0 = ok ? ld16_nt(s) : make_uint4(0, 0, 0, 0), a1 = ok ? ld16_nt(s + 4) : make_uint4(0, 0, 0, 0);
      y[u][0] = make_float4(__uint_as_float(a0.x), __uint_as_float(a0.y), __uint_as_float(a0.z), __uint_as_float(a0.w));
      y[u][1] = make_float4(__uint_as_float(a1.x), __uint_as_float(a1.y), __uint_as_float(a1.z), __uint_as_float(a1.w));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x0.x += y[u][0].x; x0.y += y[u][0].y; x0.z += y[u][0].z; x0.w += y[u][0].w;
      x1.x += y[u][1].x; x1.y += y[u][1].y; x1.z += y[u][1].z; x1.w += y[u][1].w;
    }
  }
  const float f[8] = {x0.x * sc, x0.y * sc, x0.z * sc, x0.w * sc, x1.x * sc, x1.y * sc, x1.z * sc, x1.w * sc};
  st16_nt(dqkv + (long)r * 3L * D + c, pack8(f));
}

template <int NKS, int KW, bool PERSIST>
constexpr int bwd_smem() {
  constexpr int BQ = bwd_bq<NKS, PERSIST>();
  constexpr int NH = (NKS + 3) / 4, NO = (NKS + 1) / 2, KB = 32 * KW, TILES = (BQ / 32) * NO;
  constexpr int KSPLIT = KW >= TILES ? KW / TILES : 1;
  constexpr int NTW = KSPLIT > 1 ? 1 : (TILES + KW - 1) / KW;
  return 2 * NH * BQ * ROWB + NH * KB * ROWB + (BQ / 64) * KB * ROWB + 2 * BQ * 4 + KW * BQ * 4 +
         (KSPLIT > 1 ? (KSPLIT - 1) * TILES * 64 * 16 * 4 : 0) +
         (PERSIST ? (KSPLIT > 1 ? TILES : KW) * NTW * 16 * 64 * 4 : 0);
}

int nks_for_bwd(int hd) { return nks_for(hd); }

int bwd_keys_per_block(int hd) { return nks_for_bwd(hd) > 4 ? 128 : 256; }

// Key-block mode (one workgroup per (key block, b, h), heaviest key blocks first, then a finalize
// pass over the fp32 dQ partials) by default: measured in the GPT-2 step (B=64, T=1024, hd=64;
// profiles/round2_attn_bwd_modes.txt) it beats the persistent schedule (one workgroup per (b, h)
// sweeping its key blocks, dQ summed in place) even where B*H fills the chip in whole rounds --
// the in-place read-add-store of dQ costs the persistent kernel more than the finalize pass.
// Persistent mode is used when there is a single key block (no partial sum to form).
// (The one-wave-per-SIMD key-block backward of round 3, 4 waves x 64 keys with the whole register
// file, measured 1,453 vs 1,251 us at B = 128 and was removed: PERF.md, round 3.)
int g_bwd_mode = -1;  // 0 auto, 1 force persistent, 2 force key-block (tests, MINGPT_ATTN_BWD_MODE)

bool bwd_persistent(int T, int hd) {
  if (g_bwd_mode < 0) {
    const char* e = getenv("MINGPT_ATTN_BWD_MODE");
    g_bwd_mode = e ? atoi(e) : 0;
  }
  if (g_bwd_mode) return g_bwd_mode == 1;
  return T <= bwd_keys_per_block(hd);
}

// hd = 64 key-block backward (attn_bwd64_kernel) unless MINGPT_ATTN_BWD64=0 (tests: the general
// kernel of the same arithmetic, for a bitwise comparison)
int g_bwd64 = -1;

bool use_bwd64(const AttnArgs& a) {
  if (g_bwd64 < 0) {
    const char* e = getenv("MINGPT_ATTN_BWD64");
    g_bwd64 = e ? atoi(e) : 1;
  }
  return g_bwd64 && a.hd == 64 && a.dq_part;
}

void launch_bwd64(const AttnArgs& a, hipStream_t stream) {
  constexpr int smem = 3 * 128 * ROWB + 256 * ROWB + 2 * 256 * ROWB + 2 * 128 * 4 + 2 * 8 * 128 * 4 + 16;
  static_assert(smem <= 160 * 1024, "attn_bwd64_kernel LDS budget");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_bwd64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  // one workgroup per CU (the LDS holds one), each sweeping work items (attn_bwd64_kernel)
  static int ncu[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!ncu[dev]) {
    int n = 0;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    ncu[dev] = n > 0 ? n : 256;
  }
  const int items = a.B * a.H * ((a.T + 255) / 256);
  attn_bwd64_kernel<<<items < ncu[dev] ? items : ncu[dev], 256, smem, stream>>>(a);
}

template <int NKS, int KW>
void launch_bwd(const AttnArgs& a, hipStream_t stream) {
  if constexpr (NKS == 4) {
    if (use_bwd64(a)) return launch_bwd64(a, stream);
  }
  constexpr int smem_p = bwd_smem<NKS, KW, true>(), smem_k = bwd_smem<NKS, KW, false>();
  static_assert(smem_p <= 160 * 1024 && smem_k <= 160 * 1024, "attention backward LDS budget");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_bwd_kernel<NKS, KW, true>, hipFuncAttributeMaxDynamicSharedMemorySize, smem_p);
    hipFuncSetAttribute((const void*)attn_bwd_kernel<NKS, KW, false>, hipFuncAttributeMaxDynamicSharedMemorySize, smem_k);
    attr = true;
  }
  const int nkb = (a.T + 32 * KW - 1) / (32 * KW);
  if (a.dq_part)
    attn_bwd_kernel<NKS, KW, false><<<a.B * a.H * nkb, 64 * KW, smem_k, stream>>>(a);
  else
    attn_bwd_kernel<NKS, KW, true><<<a.B * a.H, 64 * KW, smem_p, stream>>>(a);
}

}  // namespace

namespace mg {

void attention_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse,
                   const uint32_t* dmask, float* delta, float* dq, bf16_t* dqkv, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream, float* dbias) {
  (void)seed;
  AttnArgs a{};
  a.B = B; a.T = T; a.H = H; a.hd = hd; a.D = H * hd;
  a.scale_log2 = 1.4426950408889634f / sqrtf((float)hd);
  a.thr = dmask ? (uint32_t)attention_dropout_threshold(p) : 0u;
  a.dscale = attention_dropout_scale((int)a.thr);
  a.qkv = qkv; a.out = dqkv; a.lse = const_cast<float*>(lse); a.dout = dout; a.delta = delta;
  a.dq = dq; a.dqkv = dqkv; a.dmask = dmask;
  const bool persistent = bwd_persistent(T, hd);
  a.dq_part = persistent ? 0 : (long)B * T * H * hd;
  // qkv bias gradient: the K / V columns fused into the key-block kernel; the Q columns by a
  // column-sum pass over dQ after the finalize (summing them inside the finalize, a thread per
  // 8-column chunk sweeping rows, made it 146 vs 104 + 16 us at B = 64); the persistent schedule
  // takes the column-sum pass over all of dqkv
  const int D = H * hd;
  const bool fuse_db = dbias && !persistent;
  a.dbias = fuse_db ? dbias : nullptr;
  int lg = 0;
  while ((8 << lg) < hd) ++lg;
  const long nthreads = (long)B * T * H << lg;
  a.work = use_bwd64(a) ? reinterpret_cast<int*>(dq + attention_bwd_workspace_floats(B, T, H, hd) - 64) : nullptr;
  attn_bwd_pre_kernel<<<(unsigned)cdiv(nthreads, 256), 256, 0, stream>>>(dout, out, delta, B * T, T, H, hd, lg, a.work);
  switch (nks_for(hd)) {
    case 1: launch_bwd<1, 8>(a, stream); break;
    case 2: launch_bwd<2, 8>(a, stream); break;
    case 3: launch_bwd<3, 8>(a, stream); break;
    case 4: launch_bwd<4, 8>(a, stream); break;
    case 6: launch_bwd<6, 4>(a, stream); break;
    default: launch_bwd<8, 4>(a, stream); break;
  }
  if (!persistent) {
    const long n8 = (long)B * T * (H * hd / 8);
    attn_dq_finalize_kernel<<<(unsigned)cdiv(n8, 256), 256, 0, stream>>>(
        dq, dqkv, B * T, H * hd, T, bwd_keys_per_block(hd), a.dq_part, 0.6931471805599453f * a.dscale);
  }
  if (fuse_db) bias_grad(dqkv, dbias, (long)B * T, D, stream, 3L * D);  // Q columns
  else if (dbias) bias_grad(dqkv, dbias, (long)B * T, 3 * D, stream);
}

void attention_set_bwd_mode(int mode) { g_bwd_mode = mode; }

void attention_set_bwd64(int on) { g_bwd64 = on; }

#ifdef MG_BWD64_STAMPS
void attention_bwd64_stamps(unsigned long long* host) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bwd64_stamps), sizeof(g_bwd64_stamps));
  (void)hipMemcpyFromSymbol(host + 64 * 4 * 8 * 8, HIP_SYMBOL(g_bwd64_pe), sizeof(g_bwd64_pe));
}
#endif

size_t attention_bwd_workspace_floats(int B, int T, int H, int hd) {
  const size_t one = (size_t)B * T * H * hd;
  if (bwd_persistent(T, hd)) return one;
  const int kb = bwd_keys_per_block(hd);
  return one * (size_t)((T + kb - 1) / kb) + 64;  // + attn_bwd64_kernel's work counter
}

}  // namespace mg
