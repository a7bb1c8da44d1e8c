// Checks csrc/lse_fast.h against the reference's LogSumExp formula
// (unigram_model.cc:51-63, glibc double exp/log): every certified fast-path
// result must be bit-identical; prints the fallback rate.
//   g++ -O2 -std=c++17 -I tools/estep_variants tools/estep_variants/lse_fast_check.cc -o lse_fast_check
//   ./lse_fast_check [samples] [seed]
#include <cstdio>
#include <cstdlib>
#include <random>

#include "lse_fast.h"  // (tools/estep_variants: the rejected variant, kept with its checker)

using spm_amd::LseEntry;

static float RefLse(float x, float y, bool init_mode) {
  if (init_mode) return y;
  const float vmin = std::min(x, y);
  const float vmax = std::max(x, y);
  const float kMinusLogEpsilon = 50;
  if (vmax > vmin + kMinusLogEpsilon) return vmax;
  return vmax + log(exp(double(vmin - vmax)) + 1.0);
}

int main(int argc, char **argv) {
  const long long N = argc > 1 ? std::atoll(argv[1]) : 20000000;
  const unsigned seed = argc > 2 ? static_cast<unsigned>(std::atoi(argv[2])) : 1;
  const auto tab = spm_amd::MakeLseTable();
  // Sixth derivative of softplus as a polynomial in s (P_{n+1} = P_n' s(1-s)):
  // the Taylor remainder bound used in lse_fast.h.
  {
    double mx = 0;
    for (int k = 0; k <= 100000; ++k) {
      const long double s = k / 100000.0L;
      // coefficients of P_n in s, n = 1..6
      long double p[8] = {0, 1, 0, 0, 0, 0, 0, 0};  // P_1 = s
      for (int n = 1; n < 6; ++n) {
        long double dp[8] = {0}, q[9] = {0};
        for (int i = 1; i < 8; ++i) dp[i - 1] = i * p[i];
        for (int i = 0; i < 7; ++i) {  // * (s - s^2)
          q[i + 1] += dp[i];
          q[i + 2] -= dp[i];
        }
        for (int i = 0; i < 8; ++i) p[i] = q[i];
      }
      long double v = 0;
      for (int i = 7; i >= 0; --i) v = v * s + p[i];
      if (std::fabs(static_cast<double>(v)) > mx) mx = std::fabs(static_cast<double>(v));
    }
    const double rem = mx / 720.0 * std::pow(1.0 / 64, 6);
    std::printf("max|f6| %.6f  Taylor remainder <= %.3e (2^%.1f)\n", mx, rem, std::log2(rem));
    if (rem > 0x1p-46) {
      std::printf("FAIL: remainder above the budget\n");
      return 1;
    }
  }
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long long fast = 0, slow = 0, bad = 0, shortcut = 0, kslow[6] = {0}, kall[6] = {0};
  for (long long i = 0; i < N; ++i) {
    float x, y;
    const int kind = static_cast<int>(i % 6);
    if (kind == 0) {  // lattice-like: alphas of sentences, node scores
      x = static_cast<float>(-U(rng) * 300.0);
      y = static_cast<float>(x - (U(rng) - 0.3) * 30.0);
    } else if (kind == 1) {  // small magnitudes
      const double m = std::pow(2.0, -30.0 + 35.0 * U(rng));
      x = static_cast<float>(-m);
      y = static_cast<float>(-m * (1.0 + 60.0 * U(rng)));
    } else if (kind == 2) {  // wide differences up to and past 50
      x = static_cast<float>(-U(rng) * 2000.0);
      y = static_cast<float>(x - U(rng) * 60.0);
    } else if (kind == 3) {  // near-equal arguments
      x = static_cast<float>(-U(rng) * 100.0);
      const uint32_t b = spm_amd::LseFloatBits(x) + static_cast<uint32_t>(rng() % 64);
      y = spm_amd::LseBitsFloat(b);
    } else if (kind == 4) {  // positive values too (freq-weighted sums can be)
      x = static_cast<float>((U(rng) - 0.5) * 100.0);
      y = static_cast<float>((U(rng) - 0.5) * 100.0);
    } else {  // random bit patterns in a finite range
      x = spm_amd::LseBitsFloat(static_cast<uint32_t>(rng()) & 0xC3FFFFFFu);
      y = spm_amd::LseBitsFloat(static_cast<uint32_t>(rng()) & 0xC3FFFFFFu);
    }
    const float want = RefLse(x, y, false);
    const float vmin = std::min(x, y), vmax = std::max(x, y);
    if (vmax > vmin + 50.0f) {
      ++shortcut;
      continue;
    }
    float got;
    ++kall[kind];
    if (spm_amd::LseFastTry(vmax, vmin - vmax, tab.data(), &got)) {
      ++fast;
      if (spm_amd::LseFloatBits(got) != spm_amd::LseFloatBits(want)) {
        if (bad < 10) std::printf("MISMATCH x=%a y=%a got=%a want=%a\n", x, y, got, want);
        ++bad;
      }
    } else {
      ++slow;
      ++kslow[kind];
      if (spm_amd::LseFloatBits(spm_amd::LogSumExpFast(x, y, false, tab.data())) != spm_amd::LseFloatBits(want) &&
          !(want != want)) {
        if (bad < 10) std::printf("EXACT PATH MISMATCH x=%a y=%a\n", x, y);
        ++bad;
      }
    }
  }
  std::printf("samples %lld fast %lld slow %lld (rate %.3g) shortcut %lld mismatches %lld\n", N, fast, slow,
              static_cast<double>(slow) / std::max(1LL, fast + slow), shortcut, bad);
  for (int k = 0; k < 6; ++k)
    std::printf("  kind %d: fallback rate %.3g of %lld\n", k, static_cast<double>(kslow[k]) / std::max(1LL, kall[k]), kall[k]);
  std::printf("%s\n", bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
