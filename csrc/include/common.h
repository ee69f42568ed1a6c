// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//  * bf16 tensors travel as raw uint16_t bit patterns; they are loaded 8 at a time
//    (16 B per lane, the coalescing sweet spot on CDNA) and widened to fp32 with a shift.
//  * a wave is 64 lanes; block sizes are multiples of 64.
//  * every launch takes an explicit hipStream_t (the caller's current torch stream), so a
//    whole step can be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MG_DEVICE __device__ __forceinline__

namespace mg {

constexpr int kWave = 64;

typedef uint16_t bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

MG_DEVICE float bf2f(uint32_t v) { return __uint_as_float(v << 16); }

MG_DEVICE bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // gfx950: v_cvt_pk_bf16_f32, round-to-nearest-even, NaN-preserving
  return __builtin_bit_cast(bf16_t, h);
}

// ONE v_cvt_pk_bf16_f32 (two scalar converts + shift + or when written element-wise)
MG_DEVICE uint32_t pack2(float lo, float hi) {
  const f32x2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// 8 x bf16 <-> 8 x f32 through one 16-byte vector.
MG_DEVICE void unpack8(const uint4& u, float (&f)[8]) {
  f[0] = bf2f(u.x & 0xffffu); f[1] = bf2f(u.x >> 16);
  f[2] = bf2f(u.y & 0xffffu); f[3] = bf2f(u.y >> 16);
  f[4] = bf2f(u.z & 0xffffu); f[5] = bf2f(u.z >> 16);
  f[6] = bf2f(u.w & 0xffffu); f[7] = bf2f(u.w >> 16);
}

MG_DEVICE uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

MG_DEVICE uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
// non-temporal 16-byte load (streamed-once weights: decode GEMV)
MG_DEVICE uint4 ld16_nt(const void* p) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// hipGraph mode: a captured kernel's seed argument is an offset into a per-replay stream whose
// counter lives in device memory (incremented inside the graph), so every replay draws new
// dropout masks; nullptr = eager launch, the argument is the seed itself.
MG_DEVICE uint64_t eff_seed(uint64_t s, const uint64_t* ofs) {
  return ofs ? s + ofs[0] * 0x9E3779B97F4A7C15ull : s;
}

// Opaque to the optimiser: values derived from v before the fence are recomputed after it
// instead of being kept live (keeps packed bf16 packed across a reduction; see layernorm.hip).
MG_DEVICE void reg_fence(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
MG_DEVICE void st16(void* p, const uint4& v) { *reinterpret_cast<uint4*>(p) = v; }
// non-temporal 16-byte store (a large output consumed by a later kernel: keep L2 / MALL for inputs)
MG_DEVICE void st16_nt(void* p, const uint4& v) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(p));
}

// ---------------------------------------------------------------- wave / block reductions
MG_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

MG_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over a block of NW waves; `red` must hold NW floats of LDS. Result broadcast to all.
template <int NW>
MG_DEVICE float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  return t;
}

template <int NW>
MG_DEVICE float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  return t;
}

// ---------------------------------------------------------------- residual-stream dropout mask
// Exact nn.Dropout(p) decisions to 1/65536: keep iff a 16-bit uniform >= thr16 = round(65536 p),
// scale 65536 / (65536 - thr16) (p = 0.1 -> 0.100006; the 8-bit decisions of rounds 1-3 ran
// p = 0.1 as 26/256 = 0.1016).  Element (m, n) of a row-major [M, N] tensor takes half (n & 1) of
// the word  fmix32(m * ceil(N / 2) + (n >> 1) + key(seed))  (32-bit index arithmetic: exact below
// 2^32 words, i.e. 8 G elements per tensor).  One word per 2 consecutive elements: a GEMM epilogue
// lane holding C[m][n..n+3] draws two, a thread owning 8 consecutive elements four.  The murmur3
// finaliser is 2 multiplies per word (a Philox-4x32-10 generator, used in round 1, cost 40
// quarter-rate multiplies per 16 decisions and made the standalone dropout-backward kernels
// RNG-bound).  Counter-based: backward regenerates the mask, nothing is stored.
constexpr uint32_t kRowDropSalt = 0x0d0f0d0fu;

inline uint32_t dropout_threshold16(float p) {
  const double t = (double)p * 65536.0 + 0.5;
  return (uint32_t)(t < 0.0 ? 0.0 : (t > 65536.0 ? 65536.0 : t));
}
inline float dropout_scale16(uint32_t thr16) { return thr16 >= 65536u ? 0.f : 65536.f / (float)(65536u - thr16); }

MG_DEVICE uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// per-seed key (wave-uniform: scalar work)
MG_DEVICE uint32_t rowdrop_key(uint64_t seed) {
  return fmix32((uint32_t)seed ^ kRowDropSalt) ^ ((uint32_t)(seed >> 32) * 0x9E3779B1u);
}

// decision word of elements (m, n), (m, n + 1), n % 2 == 0
MG_DEVICE uint32_t rowdrop_word(uint32_t key, long m, int n, int N) {
  return fmix32((uint32_t)m * (uint32_t)((N + 1) >> 1) + (uint32_t)(n >> 1) + key);
}

// apply the mask to 2 consecutive elements whose decisions are the two halves of `word`
MG_DEVICE void rowdrop2(float* v, uint32_t word, uint32_t thr16, float scale) {
  v[0] = (word & 0xffffu) >= thr16 ? v[0] * scale : 0.f;
  v[1] = (word >> 16) >= thr16 ? v[1] * scale : 0.f;
}

// 4 consecutive elements (m, n..n+3), n % 4 == 0
MG_DEVICE void rowdrop4(float* v, uint32_t key, long m, int n, int N, uint32_t thr16, float scale) {
  rowdrop2(v, rowdrop_word(key, m, n, N), thr16, scale);
  rowdrop2(v + 2, rowdrop_word(key, m, n + 2, N), thr16, scale);
}

// 8 consecutive elements (m, n..n+7), n % 8 == 0
MG_DEVICE void rowdrop8(float (&v)[8], uint64_t seed, long m, int n, int N, uint32_t thr16, float scale) {
  const uint32_t key = rowdrop_key(seed);
  rowdrop4(v, key, m, n, N, thr16, scale);
  rowdrop4(v + 4, key, m, n + 4, N, thr16, scale);
}

// ---------------------------------------------------------------- GELU (tanh approximation)
constexpr float kGeluK0 = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kGeluK1 = 0.044715f;

// 0.5 x (1 + tanh(u)) == x * sigmoid(2u), u = K0 (x + K1 x^3): one v_exp_f32 and one v_rcp_f32
// instead of the libm tanhf (range reduction + branches), ~4x fewer instructions in the GEMM
// epilogues.  exp2 overflows to +inf for very negative x -> rcp(inf) = 0 -> gelu -> -0, as it should.
constexpr float kGeluE0 = -2.f * kGeluK0 * 1.4426950408889634f;  // -2 K0 log2(e)
constexpr float kGeluE1 = kGeluE0 * kGeluK1;

MG_DEVICE float gelu_sigmoid(float x) {  // sigmoid(2u)
  const float x2 = x * x;
  const float e = __builtin_amdgcn_exp2f(x * __builtin_fmaf(kGeluE1, x2, kGeluE0));
  return __builtin_amdgcn_rcpf(1.f + e);
}

MG_DEVICE float gelu_f(float x) { return x * gelu_sigmoid(x); }

// d/dx [x s(x)], s = sigmoid(2u): s + 2 x s (1 - s) K0 (1 + 3 K1 x^2)
MG_DEVICE float gelu_grad_from(float x, float sg) {
  return __builtin_fmaf(2.f * kGeluK0 * x * sg * (1.f - sg), __builtin_fmaf(3.f * kGeluK1, x * x, 1.f), sg);
}
MG_DEVICE float gelu_grad(float x) { return gelu_grad_from(x, gelu_sigmoid(x)); }

// GELU and GELU' of two values with packed fp32 math (v_pk_mul_f32 / v_pk_fma_f32: two lanes'
// worth per instruction; only exp2 and rcp stay per element).  Same formulas and rounding steps as
// gelu_sigmoid / gelu_grad_from; used by the GEMM epilogue, where one wave per SIMD runs ~12 VALU
// ops per element with nothing to overlap them.
MG_DEVICE void gelu2(f32x2 x, f32x2& y, f32x2& g) {
  const f32x2 x2 = x * x;
  const f32x2 t = x * (kGeluE1 * x2 + kGeluE0);
  const f32x2 d = f32x2{1.f, 1.f} + f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const f32x2 sg = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  y = x * sg;
  g = (2.f * kGeluK0) * x * sg * (f32x2{1.f, 1.f} - sg) * ((3.f * kGeluK1) * x2 + 1.f) + sg;
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace mg

// Debug builds (build_ext.py --debug => -DMG_DEBUG, loaded with MINGPT_EXT_SO): data-dependent
// indices (token ids, targets) are range-checked on the device.  A bad index is clamped to a safe
// value (no out-of-bounds access, no GPU fault) and recorded with a vector atomic in a device
// error word (hipMalloc'd, mg::debug_err_word(); nullptr in release builds, where the check
// compiles away).  The host reads and clears it after each op (mg::debug_error_bits,
// ops/_ext.py MINGPT_DEBUG_CHECKS=1) and raises naming the op.
namespace mg {
unsigned int* debug_err_word();
}
#ifdef MG_DEBUG
#define MG_CHECK_INDEX(var, ok, safe, err, bit) \
  if (!(ok)) {                                  \
    atomicOr((err), (bit));                     \
    (var) = (safe);                             \
  }
#else
#define MG_CHECK_INDEX(var, ok, safe, err, bit)
#endif
