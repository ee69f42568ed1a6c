// Shared pieces of the attention kernels (attention.hip: decode; attention_train.hip: training
// forward / backward and the dropout keep-bit generator).
#pragma once
#include "common.h"

namespace mg {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// LDS images hold 64 head-dim columns per row (128 B); a head dim > 64 is stored as two such
// 64-column halves, each its own [rows][128 B] image, so every fragment read below is the same.
constexpr int ROWB = 128;
constexpr float kNegBig = -1e30f;

// conflict-free for ds_read_b128 (32-row operand) and both ds_read_b64_tr_b16 patterns
MG_DEVICE int swz(int r) { return ((r >> 1) & 3) | ((((r >> 1) ^ (r >> 3)) & 1) << 2); }
MG_DEVICE int lds_off(int row, int ch) { return row * ROWB + ((ch ^ swz(row)) << 4); }
// byte offset of a transposed-read lane address (row, column) in an lds_off image
MG_DEVICE int tr_off(int row, int col) { return lds_off(row, col >> 3) + (col & 7) * 2; }

struct AttnArgs {
  const bf16_t* qkv;
  bf16_t* out;
  float* lse;          // [B*H*T], log2 domain of the scaled scores
  const bf16_t* dout;  // bwd
  const float* delta;  // bwd [B*H*T]
  float* dq;           // bwd fp32 dQ accumulator [B*T, D] (or per-key-block partials)
  long dq_part;        // bwd partial mode: elements between the per-key-block dQ partials (0: persistent)
  bf16_t* dqkv;        // bwd [B*T, 3D]
  const uint32_t* dmask;  // dropout keep-bits, row words (attention_train.hip, mask kernel)
  int B, T, H, hd, D;
  float scale_log2;    // log2(e) / sqrt(hd)
  uint32_t thr;        // 16-bit keep threshold: keep iff a 16-bit uniform >= thr (0 = no dropout)
  float dscale;        // 1 / (1 - thr/65536)
  float* dbias;        // bwd key-block mode: += column sums of dK / dV into [D, 3D) (qkv bias grad), or null
  int* work;           // bwd hd = 64: work-item counter (zeroed by attn_bwd_pre_kernel)
};

// 16-column MFMA k-steps a head dim is instantiated with: {1, 2, 3, 4, 6, 8}
inline int nks_for(int hd) {
  const int k = (hd + 15) / 16;
  return k <= 4 ? k : (k <= 6 ? 6 : 8);
}

MG_DEVICE float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }  // v_exp_f32, no denorm fixup

// Bit of score e (= 16 sub + r of a forward lane's 32 scores in a 64-key tile) in its dropout row
// word: the packed pair j = e >> 1 (P operand word j) at bits j (low) and 16 + j (high).
constexpr MG_DEVICE int drop_bit(int e) { return ((e & 1) << 4) + (e >> 1); }

// 32-bit avalanche mixer (xorshift-multiply, "lowbias32" constants): a bijection with good
// avalanche; the attention-dropout bytes are mix32 of distinct counters.
MG_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
inline uint32_t mix32_host(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// ------------------------------------------------------------------------------- forward
// buffer descriptor over [base + off, base + total): reads past the end return 0.  The inputs are
// readfirstlane'd so the compiler sees a uniform descriptor (no waterfall loop per load).
MG_DEVICE __amdgpu_buffer_rsrc_t kv_rsrc(const bf16_t* base, uint64_t total, uint64_t off) {
  const uint64_t p = reinterpret_cast<uint64_t>(base) + off;
  const uint64_t left = off < total ? total - off : 0;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)(left < 0xffffffffull ? left : 0xffffffffull));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

MG_DEVICE bf16x8 lds_row_at(const char* base, int o) { return *reinterpret_cast<const bf16x8*>(base + o); }

// Transposed fragment from two per-lane offsets (rows r0+q and r0+8+q, or +4): the swizzle is
// periodic in the row with period 16, so a 16-row-aligned row base is a plain byte offset the
// caller passes as a compile-time constant (it lands in the ds_read offset field).
MG_DEVICE bf16x8 lds_tr_at(const char* base, int oa, int ob) {
  const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + oa));
  const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + ob));
  const s16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// 8 consecutive accumulator values -> one bf16x8 MFMA operand (4 v_cvt_pk_bf16_f32)
MG_DEVICE bf16x8 pack_frag(const f32x16& a, int s) {
  const uint4 u = make_uint4(pack2(a[8 * s], a[8 * s + 1]), pack2(a[8 * s + 2], a[8 * s + 3]),
                             pack2(a[8 * s + 4], a[8 * s + 5]), pack2(a[8 * s + 6], a[8 * s + 7]));
  return __builtin_bit_cast(bf16x8, u);
}

// combine a value with the partner lane's (lane ^ 32) on gfx950: one v_permlane32_swap leaves
// {low-half value, high-half value} in the two results on every lane, no per-lane select
MG_DEVICE float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MG_DEVICE float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

}  // namespace attn
}  // namespace mg
