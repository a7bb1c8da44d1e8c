// A/B of the PARITY E-step record sort (estep_kernels.hip): hipcub's default
// onesweep (8-bit digits: 3 passes over 19-bit keys) against rocprim onesweep
// configs with 10-bit digits (2 passes).  Records: uint32 key = bucket * V +
// piece id (T = 16, V = 31997, ids skewed like a unigram lattice), fp64 value.
// Checks that every config yields the same (stable) permutation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_ab.hip -o /tmp/sort_ab
//   /tmp/sort_ab [records]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <unsigned Bits, unsigned HB, unsigned HI, unsigned SB, unsigned SI>
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                       rocprim::radix_sort_onesweep_config<rocprim::kernel_config<HB, HI>,
                                                                           rocprim::kernel_config<SB, SI>, Bits,
                                                                           rocprim::block_radix_rank_algorithm::match>,
                                       0>;

template <class C>
float run_rocprim(const uint32_t *k, uint32_t *k2, const double *v, double *v2, int n, int end_bit, void *&tmp,
                  size_t &cap, int reps) {
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs<C>(nullptr, tb, k, k2, v, v2, n, 0, end_bit, 0));
  if (tb > cap) { if (tmp) CK(hipFree(tmp)); CK(hipMalloc(&tmp, tb)); cap = tb; }
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(rocprim::radix_sort_pairs<C>(tmp, tb, k, k2, v, v2, n, 0, end_bit, 0));
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_pairs<C>(tmp, tb, k, k2, v, v2, n, 0, end_bit, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 150000000;
  const int T = 16, V = 31997, reps = 10;
  std::vector<uint32_t> hk(n);
  std::vector<double> hv(n);
  std::mt19937_64 g(7);
  std::geometric_distribution<int> geo(0.002);
  for (int i = 0; i < n; ++i) {
    const int sent = i / 38;  // ~38 nodes per sentence
    int id = geo(g) % V;
    hk[i] = static_cast<uint32_t>((sent % T) * V + id);
    hv[i] = static_cast<double>(i);
  }
  uint32_t *k, *k2;
  double *v, *v2;
  CK(hipMalloc(&k, n * 4ull)); CK(hipMalloc(&k2, n * 4ull));
  CK(hipMalloc(&v, n * 8ull)); CK(hipMalloc(&v2, n * 8ull));
  CK(hipMemcpy(k, hk.data(), n * 4ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), n * 8ull, hipMemcpyHostToDevice));
  int end_bit = 1;
  while ((1ull << end_bit) < static_cast<uint64_t>(T) * V) ++end_bit;
  void *tmp = nullptr;
  size_t cap = 0;
  std::vector<double> ref(n), got(n);
  // hipcub default (what estep_kernels.hip used)
  {
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k, k2, v, v2, n, 0, end_bit, 0));
    CK(hipMalloc(&tmp, tb)); cap = tb;
    CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k, k2, v, v2, n, 0, end_bit, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k, k2, v, v2, n, 0, end_bit, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(ref.data(), v2, n * 8ull, hipMemcpyDeviceToHost));
    printf("records %d end_bit %d\nhipcub default             %.3f ms  %.2f GB/s per pass-equivalent\n", n, end_bit,
           ms / reps, 24.0 * n * 3 / (ms / reps * 1e6));
  }
  auto check = [&](const char *name, float ms) {
    CK(hipMemcpy(got.data(), v2, n * 8ull, hipMemcpyDeviceToHost));
    bool eq = got == ref;
    printf("%-26s %.3f ms  same permutation: %s\n", name, ms, eq ? "yes" : "NO");
  };
  check("rocprim 10b 1024x8/1024x8", run_rocprim<Cfg<10, 1024, 8, 1024, 8>>(k, k2, v, v2, n, end_bit, tmp, cap, reps));
  check("rocprim 10b 1024x8/1024x12", run_rocprim<Cfg<10, 1024, 8, 1024, 12>>(k, k2, v, v2, n, end_bit, tmp, cap, reps));
  check("rocprim 10b 1024x16/1024x6", run_rocprim<Cfg<10, 1024, 16, 1024, 6>>(k, k2, v, v2, n, end_bit, tmp, cap, reps));
  check("rocprim 8b 1024x8/1024x8", run_rocprim<Cfg<8, 1024, 8, 1024, 8>>(k, k2, v, v2, n, end_bit, tmp, cap, reps));
  return 0;
}
