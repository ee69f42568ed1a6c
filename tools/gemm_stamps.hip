// gemm_stamps: diagnostic build of the GEMM kernels with per-phase s_memtime stamps.
// Runs one M x N x K GEMM (random bf16; layout 0 = NT forward, 1 = NN data gradient, 2 = TN weight gradient: fp32
// split-K accumulate, K = tokens) under a forced tile config and prints, per phase of
// the ping-pong kernel's K-tile MG_GEMM_STAMPS, the median cycles of each segment over all waves:
//   reads+DMA issue | vmcnt wait | barrier 1 | lgkmcnt wait | MFMA | barrier 2 (next phase start)
// Build: hipcc --offload-arch=gfx950 -O3 -DMG_GEMM_STAMPS=20 -Icsrc/include tools/gemm_stamps.hip
// (-DMG_GEMM_STAMPS=1000 -DMG_GEMM_EPI_STAMPS: W4 epilogue segments instead of a K-tile's)
#include "../csrc/kernels/gemm.hip"

namespace mg {
const uint64_t* graph_seed_ofs() { return nullptr; }  // eager launches only (adamw.hip owns it in _C.so)
}  // namespace mg

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 8192,
            K = argc > 3 ? atoi(argv[3]) : 8192, variant = argc > 4 ? atoi(argv[4]) : 4,
            layout = argc > 5 ? atoi(argv[5]) : 0;
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
  std::mt19937 rng(1);
  std::uniform_int_distribution<int> d(0, 0x7f);
  for (auto& v : ha) v = 0x3f00 | d(rng);  // bf16 in [0.5, 1): random mantissas
  for (auto& v : hb) v = 0xbf00 | d(rng);
  bf16_t *a, *b, *c;
  unsigned long long* dbg;
  hipMalloc(&a, ha.size() * 2);
  hipMalloc(&b, hb.size() * 2);
  hipMalloc(&c, (size_t)M * N * (layout == 2 ? 4 : 2));
  hipMemset(c, 0, (size_t)M * N * (layout == 2 ? 4 : 2));
  // blocks with stamp slots: output tiles x split-K chunks (at most 64 splits)
  const int blocks = cdiv(M, 256) * cdiv(N, 256) * (layout == 2 ? 64 : 1);
  hipMalloc(&dbg, (size_t)blocks * 8 * 24 * 8);
  hipMemset(dbg, 0, (size_t)blocks * 8 * 24 * 8);
  hipMemcpy(a, ha.data(), ha.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), hb.size() * 2, hipMemcpyHostToDevice);
  mg::gemm_set_variant(variant);
  auto run = [&] {
    if (layout == 2)  // C[M, N] += A[K, M]^T B[K, N]
      mg::gemm(2, 0, a, b, c, M, N, N, M, N, K, M, N, K, K, nullptr, nullptr, nullptr, 0.f, 0, 0,
               (size_t)M * K * 2, (size_t)N * K * 2);
    else if (layout == 1)  // data gradient: C[M, N] = A[M, K] B[K, N]
      mg::gemm(1, 0, a, b, c, K, N, N, M, N, K, M, N, K, K, nullptr, nullptr, nullptr, 0.f, 0, 0,
               (size_t)M * K * 2, (size_t)N * K * 2);
    else
      mg::gemm(0, 0, a, b, c, K, K, N, M, N, K, M, N, K, K, nullptr, nullptr, nullptr, 0.f, 0, 0,
               (size_t)M * K * 2, (size_t)N * K * 2);
  };
  for (int i = 0; i < 3; ++i) run();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) run();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("variant %d layout %d  %dx%dx%d: %.3f ms  %.1f TF/s\n", variant, layout, M, N, K, ms / 5,
         2.0 * M * N * K / (ms / 5 * 1e-3) / 1e12);
  mg::gemm_set_debug_buffer(dbg);
  run();
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)blocks * 8 * 24);
  hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost);
  if (variant == 5 || variant == 6) {  // W4: K-tile segments and per-tile prologue / loop / epilogue
    const char* wseg[5] = {"phaseA", "wait", "barrier", "phaseB", "fragwait"};
    auto med = [&](int k0, int k1) {
      std::vector<long long> v;
      for (int bl = 0; bl < blocks; ++bl)
        for (int w = 0; w < 4; ++w) {
          const unsigned long long* s = &h[((size_t)bl * 8 + w) * 24];
          if (s[k0] && s[k1]) v.push_back((long long)(s[k1] - s[k0]));
        }
      std::sort(v.begin(), v.end());
      return v.empty() ? -1LL : v[v.size() / 2];
    };
    printf("W4 K-tile %d, median cycles:", MG_GEMM_STAMPS);
    for (int k = 0; k < 5; ++k) printf(" %s=%lld", wseg[k], med(k, k + 1));
    printf("\nper tile: prologue=%lld main_loop=%lld epilogue=%lld (K-tiles %d)\n", med(6, 7), med(7, 8),
           med(8, 9), K / 64);
#ifdef MG_GEMM_EPI_STAMPS
    printf("epilogue: to-LDS issue=%lld LDS wait=%lld reads+stores issue=%lld store drain=%lld\n", med(8, 0),
           med(0, 1), med(1, 2), med(2, 9));
#endif
    // wall time per CU round: first start to last end over all blocks
    unsigned long long lo = ~0ull, hi = 0;
    for (int bl = 0; bl < blocks; ++bl) {
      const unsigned long long* s = &h[(size_t)bl * 8 * 24];
      if (s[6]) lo = std::min(lo, s[6]);
      if (s[9]) hi = std::max(hi, s[9]);
    }
    printf("span %llu cycles for %d tiles\n", hi - lo, blocks);
    return 0;
  }
  const char* seg[6] = {"reads+dma", "vmcnt", "barrier1", "lgkmcnt", "mfma", "barrier2"};
  for (int grp = 0; grp < 2; ++grp) {
    printf("group %d (waves %d-%d), median cycles per segment:\n", grp, grp * 4, grp * 4 + 3);
    for (int p = 0; p < 4; ++p) {
      printf("  phase %d:", p);
      for (int k = 0; k < 6; ++k) {
        std::vector<long long> v;
        for (int bl = 0; bl < blocks; ++bl)
          for (int w = grp * 4; w < grp * 4 + 4; ++w) {
            const unsigned long long* s = &h[((size_t)bl * 8 + w) * 24];
            const unsigned long long t0 = s[p * 6 + k];
            const unsigned long long t1 = k < 5 ? s[p * 6 + k + 1] : (p < 3 ? s[(p + 1) * 6] : 0);
            if (t0 && t1) v.push_back((long long)(t1 - t0));
          }
        if (v.empty()) { printf(" %s=-", seg[k]); continue; }
        std::sort(v.begin(), v.end());
        printf(" %s=%lld", seg[k], v[v.size() / 2]);
      }
      printf("\n");
    }
  }
  return 0;
}
