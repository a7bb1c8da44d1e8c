// Device helpers shared by the encode and E-step kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace spm_amd {

constexpr int kAmbEntries = 4;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Compile-time loop: f(integral_constant<int, I>) for I in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void StaticFor(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    StaticFor<B + 1, E>(f);
  }
}

__device__ __forceinline__ uint32_t OneCharLenDev(uint32_t lead) {
  // util.h:389 table "\1\1\1\1\1\1\1\1\1\1\1\1\2\2\3\4"[lead >> 4]
  return (0x4322111111111111ull >> ((lead >> 4) * 4)) & 0xFu;
}

// USER_DEFINED score: float(double(float(length) * max_score_) + 1.0)
// (unigram_model.cc:589-591: length * max_score_ + 1.0 assigned to float).
__device__ __forceinline__ float UserDefinedScore(int chars, float max_score) {
  const float prod = __fmul_rn(static_cast<float>(chars), max_score);
  return static_cast<float>(__dadd_rn(static_cast<double>(prod), 1.0));
}

// |hi - lo| small enough that fl(lo + s) == fl(hi + s) is possible for some
// node score |s| < mag (4-ulp margin at the larger magnitude).
__device__ __forceinline__ bool NearTie(float lo, float hi, float mag) {
  const float m = fmaxf(fabsf(lo), fabsf(hi)) + mag;
  return __fsub_rn(hi, lo) <= m * 4.76837158203125e-7f;  // 2^-21
}

// NearTie with the magnitude taken from hi alone: hi - lo <= (max(|lo|,|hi|)
// + mag)·2^-21 implies hi - lo <= (|hi| + mag)·2^-20, so this flags a
// superset of NearTie's pairs, and is false for lo = -inf (an empty slot).
__device__ __forceinline__ bool NearTieHi(float lo, float hi, float mag) {
  return __fsub_rn(hi, lo) <= (fabsf(hi) + mag) * 9.5367431640625e-7f;  // 2^-20
}

// LogSumExp of unigram_model.cc:51-63: float storage, double exp/log.
__device__ __forceinline__ float LogSumExpDev(float x, float y, bool init_mode) {
  if (init_mode) return y;
  const float vmin = y < x ? y : x;  // std::min
  const float vmax = x < y ? y : x;  // std::max
  if (vmax > __fadd_rn(vmin, 50.0f)) return vmax;
  return static_cast<float>(
      __dadd_rn(static_cast<double>(vmax),
                log(__dadd_rn(exp(static_cast<double>(__fsub_rn(vmin, vmax))), 1.0))));
}

}  // namespace spm_amd
