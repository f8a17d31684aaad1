// Diagnostic (not part of the library): occupancy of the ring correlation kernels as the
// runtime reports it, and a residency census of a real launch (which workgroups ran
// concurrently on the same CU).  Build: hipcc -DPWC_RING_CENSUS ... tools/occupancy.hip
#include "../pwc-net_pytorch_amd/csrc/corr_ring.hip"
#include <cstdio>
#include <algorithm>
#include <vector>

using namespace pwc;

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
  const int B = argc > 1 ? atoi(argv[1]) : 7, C = 32, H = 96, W = 112;
  size_t n = (size_t)B * C * H * W;
  float *a, *b, *o;
  (void)hipMalloc(&a, n * 4);
  (void)hipMalloc(&b, n * 4);
  (void)hipMalloc(&o, (size_t)B * 81 * H * W * 4);
  (void)hipMemset(a, 0, n * 4);
  (void)hipMemset(b, 0, n * 4);
  const int nb = B * 6 * 7;
  (void)hipMalloc(&g_census, nb * 16);
  for (int rep = 0; rep < 3; ++rep)
    (void)corr_forward_ring_f32(a, b, o, B, C, H, W, H, W, 0, 4, 2, 0, 32.f, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned> h(nb * 4);
  (void)hipMemcpy(h.data(), g_census, nb * 16, hipMemcpyDeviceToHost);
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
  for (unsigned x = 0; x < 8; ++x) {
    unsigned lo = ~0u, hi = 0, first_end = ~0u, last_start = 0;
    int cnt = 0;
    for (int i = 0; i < nb; ++i)
      if (h[i * 4 + 1] == x) {
        ++cnt;
        lo = std::min(lo, h[i * 4 + 2]);
        hi = std::max(hi, h[i * 4 + 3]);
        first_end = std::min(first_end, h[i * 4 + 3]);
        last_start = std::max(last_start, h[i * 4 + 2]);
      }
    printf("  xcc %u: %d wg, span %u ticks, last start +%u, first end +%u\n", x, cnt, hi - lo,
           last_start - lo, first_end - lo);
  }
  return 0;
}
