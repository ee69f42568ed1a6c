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
  uint32_t* dmask;     // dropout keep-bits [B*H][2*ceil(T/64)][T] (attention_train.hip writes, bwd reads)
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

// =============================================================================== decode
// One new query per sequence attending to a KV cache held as qkv rows [B, Tmax, 3D] (the prefill
// writes its qkv GEMM output straight into it).  Split-key ("flash-decoding") form: grid =
// B*H*S, workgroup (b, h, s) takes keys [s*CH, (s+1)*CH) of 0..pos, writes its partial softmax
// state (max, sum, sum p v) and the last of the S workgroups of (b, h) to finish combines them --
// a (b, h) per workgroup left the chip nearly idle (12 workgroups at B = 1) with each key's row a
// serial latency.  The hand-off between workgroups uses agent-scope atomic stores / loads for the
// partials (sc1: no cache of another CU or XCD is involved), each wave draining its stores before
// the workgroup's counter increment (MI355X_MICROARCH 'Correctness boundaries').  The last
// workgroup resets the counter, so the kernel can be replayed inside a hipGraph.
constexpr int kDecSplitsMax = 16;  // combine handles up to this many partials per (b, h)

__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16_t* __restrict__ qkv_new,
                                                          bf16_t* __restrict__ cache,
                                                          bf16_t* __restrict__ out, int H, int hd,
                                                          int D, long Tmax, int pos,
                                                          const int* __restrict__ pos_dev,
                                                          float scale_log2, int S, int CH,  // CH: set below
                                                          float* __restrict__ part,
                                                          unsigned* __restrict__ counters) {
  if (pos_dev) pos = min(max(*pos_dev, 0), (int)Tmax - 1);  // hipGraph decode: position in device memory
  __shared__ float qs[128];
  __shared__ float sc[256];
  __shared__ float red[16];
  __shared__ float acc[256 * 8];
  __shared__ int last_flag;
  const int bh = blockIdx.x / S, sp = blockIdx.x % S;
  const int b = bh / H, hh = bh % H;
  const long ld = 3L * D;
  const bf16_t* qrow = qkv_new + (long)b * ld + hh * hd;
  bf16_t* cb = cache + (long)b * Tmax * ld;
  if (sp == 0) {  // append this step's K/V at row pos (readers take row pos from qkv_new)
    for (int i = threadIdx.x; i < 2 * hd; i += 256) {
      const int which = i / hd, d = i % hd;
      cb[(long)pos * ld + (long)D * (1 + which) + hh * hd + d] = qrow[(long)D * (1 + which) + d];
    }
  }
  for (int d = threadIdx.x; d < hd; d += 256) qs[d] = bf2f(qrow[d]);
  __syncthreads();
  const int L = pos + 1;
  // splits actually used at this position: ~128 keys each (a short context is one workgroup and
  // skips the hand-off); the grid is sized for Tmax so a captured graph replays at any position
  const int Se = min(S, (L + 127) / 128);
  if (sp >= Se) return;  // never counted: the last arrival is the Se-th
  CH = (L + Se - 1) / Se;
  const int k0 = sp * CH, k1 = min(k0 + CH, L);
  const int nk = max(k1 - k0, 0);
  // scores: one key per thread (CH <= 256)
  float s = -INFINITY;
  if (threadIdx.x < nk) {
    const int j = k0 + threadIdx.x;
    const bf16_t* kr = (j == pos) ? qrow + D : cb + (long)j * ld + D + hh * hd;
    float a = 0.f;
    for (int d = 0; d < hd; d += 8) {
      float k8[8];
      unpack8(ld16(kr + d), k8);
#pragma unroll
      for (int e = 0; e < 8; ++e) a += qs[d + e] * k8[e];
    }
    s = a * scale_log2;
  }
  const float mx = block_max<4>(s, red);
  const float p = threadIdx.x < nk ? fexp2(s - mx) : 0.f;
  sc[threadIdx.x] = p;
  const float sm = block_sum<4>(p, red + 4);
  __syncthreads();
  // P V: DCH = hd/8 lanes of 8 dims per key group, 256/DCH key groups, loads issued 4 at a time
  const int dch = hd >> 3;
  const int ngrp = 256 / dch;
  const int grp = threadIdx.x / dch, d8 = (threadIdx.x % dch) * 8;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (grp < ngrp) {
    int jj = grp;
    for (; jj + 3 * ngrp < nk; jj += 4 * ngrp) {
      uint4 vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = k0 + jj + u * ngrp;
        const bf16_t* vr = (j == pos) ? qrow + 2 * D : cb + (long)j * ld + 2 * D + hh * hd;
        vv[u] = ld16(vr + d8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v8[8];
        unpack8(vv[u], v8);
        const float pj = sc[jj + u * ngrp];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pj * v8[e];
      }
    }
    for (; jj < nk; jj += ngrp) {
      const int j = k0 + jj;
      const bf16_t* vr = (j == pos) ? qrow + 2 * D : cb + (long)j * ld + 2 * D + hh * hd;
      float v8[8];
      unpack8(ld16(vr + d8), v8);
      const float pj = sc[jj];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pj * v8[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[threadIdx.x * 8 + e] = o[e];
  __syncthreads();
  if (Se == 1) {  // the whole context in this workgroup: normalise and write
    if (threadIdx.x < hd) {
      const int c = threadIdx.x / 8, e = threadIdx.x % 8;
      float v = 0.f;
      for (int g = 0; g < ngrp; ++g) v += acc[(g * dch + c) * 8 + e];
      out[(long)b * D + hh * hd + threadIdx.x] = f2bf(v / sm);
    }
    return;
  }
  // partial state of this split: {max, sum, o[hd]} (fp32)
  float* mine = part + (long)blockIdx.x * (hd + 2);
  if (threadIdx.x < hd) {
    const int c = threadIdx.x / 8, e = threadIdx.x % 8;
    float v = 0.f;
    for (int g = 0; g < ngrp; ++g) v += acc[(g * dch + c) * 8 + e];
    __hip_atomic_store(mine + 2 + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(mine, nk ? mx : -INFINITY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, sm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counters + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = prev == (unsigned)(Se - 1);
  }
  __syncthreads();
  if (!last_flag) return;
  // last split of (b, h): combine the S partial states (agent-scope loads: never a stale line),
  // every load issued before any is used
  const float* pb = part + (long)bh * S * (hd + 2);
  if (threadIdx.x < Se) {
    red[threadIdx.x] = __hip_atomic_load(pb + threadIdx.x * (hd + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sc[threadIdx.x] = __hip_atomic_load(pb + threadIdx.x * (hd + 2) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    float ov[kDecSplitsMax];
#pragma unroll
    for (int t = 0; t < kDecSplitsMax; ++t)
      ov[t] = t < Se ? __hip_atomic_load(pb + t * (hd + 2) + 2 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
    float M = -INFINITY;
    for (int t = 0; t < Se; ++t) M = fmaxf(M, red[t]);
    float Ls = 0.f, Os = 0.f;
#pragma unroll
    for (int t = 0; t < kDecSplitsMax; ++t) {
      if (t < Se && red[t] != -INFINITY) {
        const float w = fexp2(red[t] - M);
        Ls += w * sc[t];
        Os += w * ov[t];
      }
    }
    out[(long)b * D + hh * hd + threadIdx.x] = f2bf(Os / Ls);
  }
  if (threadIdx.x == 0) __hip_atomic_store(counters + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

namespace mg {

// persistent decode workspace: per-split partial states and per-(b, h) counters (zeroed once;
// the kernel leaves them zero), grown on demand outside graph capture (the warm-up step runs first)
static float* g_dec_part = nullptr;
static unsigned* g_dec_cnt = nullptr;
static size_t g_dec_part_n = 0, g_dec_cnt_n = 0;

void attention_decode(const bf16_t* qkv_new, bf16_t* cache, bf16_t* out, int B, int H, int hd,
                      long Tmax, int pos, hipStream_t stream, const int* pos_dev) {
  // fixed grid (graph replays move pos only); the kernel uses ceil(L / 128) of the S splits, so
  // each holds <= 256 keys for Tmax <= 4096 (checked by the binding)
  const int S = kDecSplitsMax;
  const int CH = 0;
  const size_t np = (size_t)B * H * S * (hd + 2), nc = (size_t)B * H;
  if (np > g_dec_part_n) {
    if (g_dec_part) hipFree(g_dec_part);
    hipMalloc(&g_dec_part, np * sizeof(float));
    g_dec_part_n = np;
  }
  if (nc > g_dec_cnt_n) {
    if (g_dec_cnt) hipFree(g_dec_cnt);
    hipMalloc(&g_dec_cnt, nc * sizeof(unsigned));
    hipMemset(g_dec_cnt, 0, nc * sizeof(unsigned));
    hipDeviceSynchronize();
    g_dec_cnt_n = nc;
  }
  attn_decode_kernel<<<B * H * S, 256, 0, stream>>>(qkv_new, cache, out, H, hd, H * hd, Tmax, pos, pos_dev,
                                                    1.4426950408889634f / sqrtf((float)hd), S, CH,
                                                    g_dec_part, g_dec_cnt);
}

}  // namespace mg
