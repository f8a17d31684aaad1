// Diagnostic (not part of the library): occupancy of the ring correlation kernels as the
// runtime reports it, and a residency census of a real launch (which workgroups ran
// concurrently on the same CU).  Build: hipcc -DPWC_RING_CENSUS ... tools/occupancy.hip
#include "../pwc-net_pytorch_amd/csrc/corr_ring.hip"
#include <cstdio>
#include <algorithm>
#include <vector>

using namespace pwc;

namespace pwc {  // the library's measurement hook lives in capi.hip; not linked here
void take_launch_events(hipEvent_t* a, hipEvent_t* b) { *a = *b = nullptr; }
}  // namespace pwc

template <class G>
void report(const char* name) {
  int n = 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_fwd_ring<G>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, corr_fwd_ring<G>, G::THREADS,
                                                     G::LDS_BYTES);
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&corr_fwd_ring<G>));
  printf("%s: threads %d lds %d numRegs %d -> API blocks/CU %d\n", name, G::THREADS,
         G::LDS_BYTES, a.numRegs, n);
}

int main(int argc, char** argv) {
  report<RingA>("RingA");
  report<RingB>("RingB");
  report<RingC>("RingC");
  const int B = argc > 1 ? atoi(argv[1]) : 7;
  const int C = argc > 3 ? atoi(argv[3]) : 32, H = argc > 4 ? atoi(argv[4]) : 96,
            W = argc > 5 ? atoi(argv[5]) : 112, maxs = argc > 6 ? atoi(argv[6]) : 1;
#ifdef PWC_RING_ABLATION
  {
    const int abl = argc > 2 ? atoi(argv[2]) : 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ablation), &abl, sizeof(int));
    printf("ablation %d\n", abl);
  }
#endif
  size_t n = (size_t)B * C * H * W;
  float *a, *b, *o;
  (void)hipMalloc(&a, n * 4);
  (void)hipMalloc(&b, n * 4);
  (void)hipMalloc(&o, (size_t)B * 81 * H * W * 4);
  (void)hipMemset(a, 0, n * 4);
  (void)hipMemset(b, 0, n * 4);
  const long long tiles = (long long)B * ((H + 15) / 16) * ((W + 15) / 16);
  const int ns = corr_pick_splits(tiles, (C + 3) / 4, maxs);
  const int nb = (int)tiles * ns;
  printf("B=%d C=%d %dx%d: %lld tiles x %d splits\n", B, C, H, W, tiles, ns);
  float* part = nullptr;
  if (maxs > 1) (void)hipMalloc(&part, (size_t)maxs * B * 81 * H * W * 4);
  (void)hipMalloc(&g_census, nb * 32);
  for (int rep = 0; rep < 3; ++rep)
    (void)corr_forward_ring_f32(a, b, o, B, C, H, W, H, W, 0, 4, 2, 0, 32.f, maxs, part, 0);
  (void)hipDeviceSynchronize();
  {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int rep = 0; rep < 50; ++rep)
      (void)corr_forward_ring_f32(a, b, o, B, C, H, W, H, W, 0, 4, 2, 0, 32.f, maxs, part, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("  back-to-back: %.2f us per launch\n", ms * 1000 / 50);
  }
  std::vector<unsigned> h8(nb * 8), h(nb * 4);
  (void)hipMemcpy(h8.data(), g_census, nb * 32, hipMemcpyDeviceToHost);
  {
    std::vector<unsigned> pro, loop, rt;
    for (int i = 0; i < nb; ++i) {
      for (int k = 0; k < 4; ++k) h[i * 4 + k] = h8[i * 8 + k];
      pro.push_back(h8[i * 8 + 4]);
      loop.push_back(h8[i * 8 + 5]);
      rt.push_back(h8[i * 8 + 6]);
    }
    std::sort(pro.begin(), pro.end());
    std::sort(loop.begin(), loop.end());
    std::sort(rt.begin(), rt.end());
    printf("  prologue cycles p50 %u | stage-loop cycles p50 %u max %u | loop ticks p50 %u -> "
           "clock %.2f GHz\n", pro[nb / 2], loop[nb / 2], loop[nb - 1], rt[nb / 2],
           (double)loop[nb / 2] / (rt[nb / 2] * 10.0));
  }
  int maxc = 0;
  double life = 0;
  unsigned tmin = ~0u, tmax = 0;
  for (int i = 0; i < nb; ++i) {
    int c = 0;
    unsigned ki = (h[i * 4] >> 8) & 0xff, xi = h[i * 4 + 1];
    life += h[i * 4 + 3] - h[i * 4 + 2];
    for (int j = 0; j < nb; ++j) {
      unsigned kj = (h[j * 4] >> 8) & 0xff, xj = h[j * 4 + 1];
      if (ki == kj && xi == xj && h[j * 4 + 2] < h[i * 4 + 3] && h[i * 4 + 2] < h[j * 4 + 3]) ++c;
    }
    if (c > maxc) maxc = c;
  }
  printf("ring B=%d (%d workgroups): max co-resident on one CU = %d, mean lifetime %.0f ticks\n",
         B, nb, maxc, life / nb);
  unsigned g0 = ~0u;
  for (int i = 0; i < nb; ++i) g0 = std::min(g0, h[i * 4 + 2]);
  std::vector<unsigned> st, en;
  for (int i = 0; i < nb; ++i) { st.push_back(h[i * 4 + 2] - g0); en.push_back(h[i * 4 + 3] - g0); }
  std::vector<unsigned> s2 = st, e2 = en;
  std::sort(s2.begin(), s2.end());
  std::sort(e2.begin(), e2.end());
  printf("  (100 MHz ticks) start: min %u p50 %u p90 %u max %u | end: min %u p50 %u max %u\n",
         s2[0], s2[nb / 2], s2[nb * 9 / 10], s2[nb - 1], e2[0], e2[nb / 2], e2[nb - 1]);
  int late = 0;
  for (int i = 0; i < nb; ++i) late += st[i] > 50;  // started > 0.5 us after the first block
  printf("  blocks starting > 0.5 us late: %d of %d\n", late, nb);
  return 0;
}
