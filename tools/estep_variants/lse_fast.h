// LogSumExp of the lattice (unigram_model.cc:51-63) with a certified fast path.
//
// The reference computes, for vmax = max(x, y), vmin = min(x, y) (floats),
//   d = RN_f(vmin - vmax)                      (float subtraction)
//   r = RN_f(RN_d(vmax + log(exp(d) + 1.0)))   (double exp/log, then float)
// unless vmax > vmin + 50.  The exact restatement (LogSumExpDev,
// device_common.h) runs a double exp and a double log per call: ~100 fp64
// instructions, the largest single cost of both E-step walks.
//
// Fast path.  L = log(exp(d) + 1) is softplus(d) up to double roundings
// (|error| <= 2^-50 for d <= 0).  softplus is evaluated from a table of
// (softplus(c_j), sigmoid(c_j)) at c_j = -36 + j/32 (j = 0..1152) by its
// degree-5 Taylor polynomial around the nearest c_j, |h| <= 1/64; the
// derivatives are polynomials in sigma = sigmoid(c_j):
//   f' = s, f'' = a = s(1-s), f''' = a(1-2s), f'''' = a(1-6s+6s^2),
//   f^(5) = a(1-2s)(1-12s+12s^2);
// the truncation term is below 2^-47.5 (|f^(6)| <= 1/4), the table is built in
// long double.  For d < -36, softplus(d) < 2^-51 and L is taken as 0.
// With y = RN_d(vmax + L_approx) and r = RN_f(y), every value within
// E = 2^-42 + |y| 2^-50 of y rounds (through double, then float) to r when
// [y - E, y + E] lies strictly between the midpoints of r and its two float
// neighbours; the reference's RN_d(vmax + L) is such a value, so r is the
// reference's result.  Otherwise (a value near a rounding boundary,
// probability ~2^-20 per call at |vmax| ~ 10, or r = 0 / not finite, or NaN
// input) the caller runs the exact double formula.
// tests/test_lse_fast_cpu.py checks the fast path against the glibc formula.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#include <vector>

#if defined(__HIPCC__)
#define SPM_LSE_HD __host__ __device__ __forceinline__
#else
#define SPM_LSE_HD inline
#endif

namespace spm_amd {

struct LseEntry {
  double f0;   // softplus(c_j)
  double sig;  // sigmoid(c_j)
};

constexpr int kLseTableLo = -36;  // c_0
constexpr int kLseTableStep = 32;  // entries per unit of d
constexpr int kLseTableSize = -kLseTableLo * kLseTableStep + 1;

SPM_LSE_HD uint32_t LseFloatBits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

SPM_LSE_HD float LseBitsFloat(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// The fast path: true and *out = the reference's LogSumExp when certified.
// vmax > vmin + 50 and init_mode are the caller's (as in the reference).
SPM_LSE_HD bool LseFastTry(float vmax, float d, const LseEntry *__restrict__ tab, float *out) {
  double L;
  if (d >= static_cast<float>(kLseTableLo)) {
    const double u = (static_cast<double>(d) - kLseTableLo) * kLseTableStep;  // exact
    const double jr = std::rint(u);
    const int j = static_cast<int>(jr);
    const double h = static_cast<double>(d) - (jr * (1.0 / kLseTableStep) + kLseTableLo);  // exact
    const LseEntry e = tab[j];
    const double s = e.sig;
    const double a = std::fma(-s, s, s);                     // s(1-s)
    const double t = std::fma(-2.0, s, 1.0);                 // 1-2s
    const double q1 = std::fma(s, std::fma(6.0, s, -6.0), 1.0);    // 1-6s+6s^2
    const double q2 = std::fma(s, std::fma(12.0, s, -12.0), 1.0);  // 1-12s+12s^2
    const double f3 = a * t;
    const double c5 = f3 * q2 * (1.0 / 120.0);
    const double c4 = a * q1 * (1.0 / 24.0);
    const double c3 = f3 * (1.0 / 6.0);
    const double c2 = a * 0.5;
    double p = std::fma(h, c5, c4);
    p = std::fma(h, p, c3);
    p = std::fma(h, p, c2);
    p = std::fma(h, p, s);
    L = std::fma(h, p, e.f0);
  } else if (d < static_cast<float>(kLseTableLo)) {
    L = 0.0;  // softplus(d) < 2^-51, inside the error bound
  } else {
    return false;  // NaN
  }
  const double y = static_cast<double>(vmax) + L;
  const float r = static_cast<float>(y);
  const uint32_t rb = LseFloatBits(r);
  const uint32_t mag = rb & 0x7FFFFFFFu;
  if (mag == 0 || mag >= 0x7F000000u) return false;  // zero, huge, inf, NaN: exact path
  // Float neighbours: one ulp up and down in value.
  const bool neg = (rb >> 31) != 0;
  const float r_up = LseBitsFloat(neg ? rb - 1 : rb + 1);
  const float r_dn = LseBitsFloat(neg ? rb + 1 : rb - 1);
  const double rd = static_cast<double>(r);
  const double mid_up = (rd + static_cast<double>(r_up)) * 0.5;  // exact
  const double mid_dn = (rd + static_cast<double>(r_dn)) * 0.5;
  const double E = 0x1p-42 + std::fabs(y) * 0x1p-50;
  if (y + E < mid_up && y - E > mid_dn) {
    *out = r;
    return true;
  }
  return false;
}

// The reference formula (unigram_model.cc:51-63) for the non-certified cases.
SPM_LSE_HD float LseExact(float vmax, float d) {
  return static_cast<float>(static_cast<double>(vmax) + std::log(std::exp(static_cast<double>(d)) + 1.0));
}

// LogSumExp(x, y, init_mode) of the reference, bit-exact.
SPM_LSE_HD float LogSumExpFast(float x, float y, bool init_mode, const LseEntry *__restrict__ tab) {
  if (init_mode) return y;
  const float vmin = y < x ? y : x;  // std::min
  const float vmax = x < y ? y : x;  // std::max
  if (vmax > vmin + 50.0f) return vmax;
  const float d = vmin - vmax;
  float r;
  if (!LseFastTry(vmax, d, tab, &r)) r = LseExact(vmax, d);
  return r;
}

// The table (host code), in long double (64-bit mantissa): |error| ~2^-63.
inline std::vector<LseEntry> MakeLseTable() {
  std::vector<LseEntry> t(kLseTableSize);
  for (int j = 0; j < kLseTableSize; ++j) {
    const long double c = static_cast<long double>(kLseTableLo) + static_cast<long double>(j) / kLseTableStep;
    t[j].f0 = static_cast<double>(log1pl(expl(c)));
    t[j].sig = static_cast<double>(1.0L / (1.0L + expl(-c)));
  }
  return t;
}

}  // namespace spm_amd
