// Unigram trainer E-step for gfx950 (MI355X).
//
// Reference: unigram::Trainer::RunEStep (unigram_model_trainer.cc:237-287):
// per sentence SetSentence + TrainerModel::PopulateNodes + Lattice::
// PopulateMarginal (unigram_model.cc:272-328) + Viterbi().size(); thread n
// takes sentences i ≡ n (mod T) and sums into its own float vector, the T
// vectors are then summed in thread order.
//
// Position-level restatement used by the fast kernels.  In PopulateMarginal
//   alpha[r] = LSE_{l in end_nodes[pos(r)]} (score[l] + alpha[l])
// depends only on pos(r), and
//   beta[l]  = LSE_{r in begin_nodes[end(l)]} (score[r] + beta[r])
// only on end(l).  So per char position p the kernels keep one float
//   A[p] (alpha of every node beginning at p) and Bt[p] (beta of every node
// ending at p), accumulated in exactly the reference order:
//   estep_forward_kernel   ascending positions; nodes pushed into a register
//                          ring by char distance (end_nodes order = begin
//                          ascending); also the Viterbi count (same ring
//                          scheme as unigram_fast_kernel) and Z = A[len];
//                          A[p] goes to a per-byte float buffer.
//   estep_backward_kernel  descending positions, walking each position's
//                          begin_nodes (ascending length, then UNK) over a
//                          second ring; contribution of node (b,e):
//                          freq * exp(((A[b] + s) + Bt[e]) - Z)  (float
//                          exponent, double exp, exactly as :318-325).
// Accumulation modes:
//   FAST   : fp64 atomics into acc[V]; obj, ntok reduced in fp64 / int64.
//   PARITY : one record (bucket*V + id, fp64 contribution) per node, written
//            in the reference's per-bucket order (sentence asc, pos asc,
//            begin_nodes order); a stable radix sort by key followed by one
//            thread per (bucket, id) doing e = (float)((double)e + c) in order
//            reproduces `expected[n][id] += freq * exp(...)` bit for bit
//            (up to device vs glibc exp/log ulp differences).
// Sentences the fast kernels cannot handle exactly (near-tie chains in the
// Viterbi count, trie leaves inside a UTF-8 char, malformed UTF-8) run through
// estep_general_kernel, the reference lattice literally.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spm_hip.h"
#include "device_common.h"
#include "device_model.h"
#include "double_array.h"
#include "kernels.h"
#include "normalizer.h"
#include "trace.h"

namespace spm_amd {
constexpr int kHotPieces = 4096;
}

struct spm_hip_pieces {
  spm_amd::DoubleArray trie;
  uint64_t V = 0;
  float min_score = FLT_MAX;
  float unk_score = 0.f;
  float tie_mag = 0.f;
  uint32_t root_base = 0;
  int ring_width = 0;
  int trie_results_size = 0;
  spm_amd::DevBuf d_units, d_values, d_scores, d_vscore, d_uvs, d_uvis, d_hot_slot, d_hot_id;
  // work buffers
  spm_amd::DevBuf w_A, w_Z, w_N, w_ntok, w_flag, w_status, w_recoff, w_cnt, w_seg, w_tmp, w_scratch,
      w_bp, w_red, w_objq;
  // PARITY: records (key, value) and the sorted keys; the fold of chunk c
  // runs on fold_st while chunk c+1's walks run on the caller's stream, so
  // what the fold reads is double-buffered (set = chunk parity).
  spm_amd::DevBuf w_keys, w_vals, w_keys2;
  spm_amd::DevBuf w_svals[2], w_sseg[2], w_sobjq[2], w_heavy[2], w_light[2], w_cls[2];
  hipStream_t fold_st = nullptr;
  hipEvent_t ev_ready[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  bool ev_used[2] = {false, false};
  uint64_t fold_chunks = 0;
  uint32_t *pinned = nullptr;
  // The forward pass of pieces whose TrainerModel encodes with the byte
  // kernel runs that kernel's E-step mode (null: estep_forward_kernel).
  spm_hip_model *enc = nullptr;
  bool enc_tried = false;
  int forward_mode = 0;  // spm_hip_pieces_set_forward: 0 auto, 1 byte kernel, 2 estep_forward_kernel
  std::string enc_bytes;  // the piece list, kept to build `enc` on first use
  std::vector<uint64_t> enc_off;
  std::vector<float> enc_scores;
  spm_amd::DevBuf w_ectl;
  // PARITY record drop (estep_threshold_kernel): per-chunk bound exponents,
  // records kept per sentence, their scan and the dense kept records.  A
  // negative sentence freq ever seen turns the drop off for good (the bound
  // needs accumulators that never decrease).
  spm_amd::DevBuf w_drop, w_kept, w_koff, w_ckeys, w_cvals;
  // Tile-transposed alpha, lane maps and records (EArgs::AT / RT).
  spm_amd::DevBuf w_AT, w_lanemap, w_colmap, w_RT;
  bool neg_freq_seen = false;
  // No accumulate call since the piece set was made or last finalized: the
  // next call's first chunk drops nothing (its bounds are all zero).
  bool fresh_acc = true;
  uint64_t rec_total = 0, rec_kept = 0;  // records written / kept (spm_hip_estep_record_stats)
  // spm_hip_pieces_set_timing: HIP events around each chunk's forward and
  // backward passes on the caller's stream (groups of 4), read and released
  // by spm_hip_estep_kernel_times.
  bool timing = false;
  std::vector<hipEvent_t> tev;
  std::string last_error;
  // One E-step at a time per piece set: the work buffers above are shared by
  // the accumulate/finalize calls (RunEStep is const but single-caller).
  std::recursive_mutex mu;
};

namespace spm_amd {
namespace {

constexpr int kEBlock = 256;
constexpr uint32_t kRTRows = 32;  // tile-transposed records kept per lane (EArgs::RT)

// A/B knobs of the E-step launch (read once per process).
struct EStepKnobs {
  // SPM_HIP_ESTEP_PAIR=1: two positions per lane in flight (slower: the
  // kernel is VALU-heavy, and the pair costs 3 waves and spills).
  bool pair = false;
  // SPM_HIP_ESTEP_ROLL=0: per-depth node emission instead of the rolled
  // per-lane loop (c4 FAST 0.274 -> 0.249, PARITY 0.290 -> 0.266 s/epoch
  // with the rolled one, profiles/r04h_estep_roll_ab.txt).
  bool roll = true;
  // SPM_HIP_ESTEP_STAGE=1: deferred PARITY records staged in LDS and written
  // as one run per lane and flush (PMC writes of the backward kernel 3.48 ->
  // 1.29 GB per launch at the 12.5 M-sentence epoch, but 23 spilled VGPRs
  // instead of 14 and PARITY 0.2628 -> 0.264-0.267 s/epoch, gpurun_out/r05c).
  bool stage = false;
  // SPM_HIP_ESTEP_AT=0 / SPM_HIP_ESTEP_RT=0: alpha / deferred records in
  // their range layout instead of tile-transposed (EArgs::AT / RT).
  bool transposed_alpha = true;
  bool transposed_records = true;
};

const EStepKnobs &Knobs() {
  static const EStepKnobs k = [] {
    auto flag = [](const char *name, bool dflt) {
      const char *e = std::getenv(name);
      return e ? std::atoi(e) != 0 : dflt;
    };
    EStepKnobs x;
    x.pair = flag("SPM_HIP_ESTEP_PAIR", false);
    x.roll = flag("SPM_HIP_ESTEP_ROLL", true);
    x.stage = flag("SPM_HIP_ESTEP_STAGE", false);
    x.transposed_alpha = flag("SPM_HIP_ESTEP_AT", true);
    x.transposed_records = flag("SPM_HIP_ESTEP_RT", true);
    return x;
  }();
  return k;
}
// Accumulate calls of at least this many sentences use the byte kernel's
// E-step mode (its TrainerModel build costs ~0.1 s per piece list).
constexpr uint64_t kByteForwardMinSentences = 1ull << 20;

// PARITY record sort: onesweep, 10 bits per pass (tools/sort_ab.hip A/B).
using RecordSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 6>, 10,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

struct ToU64E {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};
constexpr int kELdsBp = 64;
constexpr int kHot = kHotPieces;  // FAST mode: per-block fp64 LDS accumulators for the hottest pieces

struct EArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  const int64_t *__restrict__ freq;
  uint64_t n;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;
  const float *__restrict__ scores;
  const float *__restrict__ vscore;  // per unit: the leaf's piece score
  // The walks' gathers: per unit (unit, score bits) for the forward pass and
  // (unit, piece id, score bits, 0) for the backward pass, so one load per
  // trie step also brings what a leaf needs (the walks are bound by the
  // vector-memory address path, not by the bytes a gather returns).
  const uint2 *__restrict__ uvs;
  const uint4 *__restrict__ uvis;
  uint32_t root_base;
  uint32_t num_units;  // entries of uvs / uvis
  float unk_score;
  float tie_mag;
  uint32_t V;
  // per-byte / per-sentence work
  float *__restrict__ A;          // alpha per byte position
  float *__restrict__ Zlat;       // lattice Z per sentence
  uint32_t *__restrict__ N;       // node count per sentence
  uint32_t *__restrict__ ntok;    // Viterbi size per sentence
  uint8_t *__restrict__ gbp;      // back-pointers beyond kELdsBp
  uint32_t *__restrict__ flagged;
  uint32_t *__restrict__ status;  // [0] flagged, [1] max flagged bytes
  // accumulation
  int mode;
  int T;
  uint64_t index_base, index_stride;
  const uint64_t *__restrict__ rec_off;
  uint32_t *__restrict__ keys;
  double *__restrict__ vals;
  double *__restrict__ acc;       // FAST: expected (fp64)
  double *__restrict__ acc_obj;   // FAST: obj (fp64)
  int64_t *__restrict__ ntok_b;   // per bucket (PARITY) or [0] (FAST)
  const int16_t *__restrict__ hot_slot;  // FAST: LDS slot of the kHot highest-score pieces, -1 else
  const int32_t *__restrict__ hot_id;    // FAST: piece id of each LDS slot
  float all_freq_f;
  // PARITY record drop (estep_threshold_kernel): per hot slot, the smallest
  // biased float exponent of the accumulators the call touches (0 = none),
  // and per sentence the records kept (written at the end of its range).
  const uint8_t *__restrict__ drop_exp;
  uint32_t *__restrict__ kept;
  // PARITY records stored with nontemporal hints (SPM_HIP_ESTEP_NT): they are
  // read back only by later kernels, so they need not displace the trie's
  // lines in L2.
  int nt;
  // Deferred record values (set while the record drop is active): a record
  // holds the float exponent ex of c = freq * exp(ex) instead of c (in the
  // vals buffer's storage), estep_compact_records_kernel computes c for the
  // kept ones only, and the drop test decides most records from ex alone.
  float *__restrict__ exs;
  // Tile-transposed alpha from the byte-kernel forward pass (kernels.h
  // EStepForwardOut::AT; null: A only): the backward pass takes the forward's
  // lane assignment (lanemap) and reads alpha of positions < kATRows from AT.
  const float *__restrict__ AT;
  const uint8_t *__restrict__ lanemap;
  // PARITY deferred records, tile-transposed: the k-th record a lane keeps
  // (k = 0 is the last slot of its sentence's range) goes to
  // RT[(tile * rt_rows + k) * 256 + lane] while k < rt_rows, later ones to
  // their range slot; estep_compact_records_kernel reads both.
  uint2 *__restrict__ RT;
  uint32_t rt_rows;
  uint16_t *__restrict__ colmap;  // (RT) lane of each sentence; 0xFFFF: records in range slots
};

// One PARITY record (key, fp64 contribution) at slot w.
__device__ __forceinline__ void StoreRecord(const EArgs &a, uint64_t w, uint32_t key, double c) {
  if (a.nt) {
    __builtin_nontemporal_store(key, a.keys + w);
    __builtin_nontemporal_store(c, a.vals + w);
  } else {
    a.keys[w] = key;
    a.vals[w] = c;
  }
}

// A deferred record (key, ex) at slot w.
__device__ __forceinline__ void StoreRecordEx(const EArgs &a, uint64_t w, uint32_t key, float ex) {
  if (a.nt) {
    __builtin_nontemporal_store(key, a.keys + w);
    __builtin_nontemporal_store(ex, a.exs + w);
  } else {
    a.keys[w] = key;
    a.exs[w] = ex;
  }
}

// The PARITY record of one node, written at --w unless dropped: its value is
// c = (double)freq * exp((double)ex) (unigram_model_trainer.cc:318-325
// restated), dropped when texp != 0 and c < 2^(texp - 152) (a quarter ulp of
// its accumulator's lower bound, estep_threshold_kernel).  With deferred
// values the test runs on ex: L = ln(2^(texp - 152) / freq) in float is
// within 2^-15 of the true bound, so ex below L - 2^-10 is dropped and ex
// above L + 2^-10 kept without computing c (exp's own error is ~2^-52
// relative); only ex inside the band (or NaN) computes c and tests it
// exactly.  lfreq = logf(freq).
// The deferred-value drop test (a.exs set): false = provably a no-op record.
__device__ __forceinline__ bool DeferredKeep(float ex, float freq_f, float lfreq, uint32_t texp) {
  if (texp) {
    constexpr float kBand = 1.0f / 1024;
    const float L = __fsub_rn(__fmul_rn(static_cast<float>(static_cast<int>(texp) - 152), 0.693147182f), lfreq);
    if (ex < __fsub_rn(L, kBand)) return false;
    if (!(ex > __fadd_rn(L, kBand))) {
      const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
      if (static_cast<uint64_t>(__double_as_longlong(c)) >> 52 < texp + 871u) return false;
    }
  }
  return true;
}

__device__ __forceinline__ void ParityRecord(const EArgs &a, uint64_t &w, uint32_t key, float ex, float freq_f,
                                             float lfreq, uint32_t texp) {
  if (a.exs) {
    if (!DeferredKeep(ex, freq_f, lfreq, texp)) return;
    --w;
    StoreRecordEx(a, w, key, ex);
    return;
  }
  const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
  // c >= 0 here (the drop is off once a negative freq is seen); NaN and
  // negative values never pass the test.
  if (texp && static_cast<uint64_t>(__double_as_longlong(c)) >> 52 < texp + 871u) return;
  --w;
  StoreRecord(a, w, key, c);
}

__device__ __forceinline__ uint32_t BucketOf(const EArgs &a, uint64_t i) {
  return static_cast<uint32_t>((a.index_base + i * a.index_stride) % static_cast<uint64_t>(a.T));
}

// Is a a structurally valid UTF-8 split?  (Backward iteration needs char
// starts == non-continuation bytes.)
__device__ __forceinline__ bool ContinuationByte(uint32_t c) { return (c & 0xC0u) == 0x80u; }

// The block's sentences are consecutive, so their bytes are one contiguous
// range: it is staged in LDS with coalesced dword loads, and the walks'
// byte reads (on the dependent chain: lead byte -> char length -> next byte)
// hit LDS instead of L1/L2.  Bytes past kEStage stay in global memory.
constexpr uint32_t kEStage = 12288;

// Lane -> sentence of the block in ascending byte length (LDS counting sort
// over 256 length buckets), so a wave's 64 lanes run similar trip counts.
__device__ __forceinline__ uint32_t SortedLane(const EArgs &a, uint64_t blk, uint32_t *hist) {
  uint32_t *perm = hist + kEBlock;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t ii = blk + tid;
  const uint32_t len = ii < a.n ? static_cast<uint32_t>(a.off[ii + 1] - a.off[ii]) : 0u;
  const uint32_t bucket = len < kEBlock - 1 ? len : kEBlock - 1;
  hist[tid] = 0;
  __syncthreads();
  const uint32_t r = atomicAdd(&hist[bucket], 1u);
  __syncthreads();
  if (wave == 0) {  // exclusive scan of 256 bins, 4 per lane
    uint32_t v[4], tot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = hist[lane * 4 + q];
      tot += v[q];
    }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    uint32_t run = x - tot;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t c = v[q];
      hist[lane * 4 + q] = run;
      run += c;
    }
  }
  __syncthreads();
  perm[hist[bucket] + r] = static_cast<uint32_t>(tid);
  __syncthreads();
  return perm[tid];
}

__device__ __forceinline__ uint64_t StageBlockBytes(const EArgs &a, uint64_t blk, uint32_t *lds,
                                                    uint64_t total) {
  const uint64_t b_0 = a.off[blk];
  const uint64_t b_1 = a.off[blk + kEBlock < a.n ? blk + kEBlock : a.n];
  const uint64_t al = b_0 & ~3ull;
  uint64_t nw = (b_1 - al + 3) / 4;
  if (nw > kEStage / 4) nw = kEStage / 4;
  for (uint64_t k = threadIdx.x; k < nw; k += kEBlock) {
    const uint64_t g = al + 4 * k;
    uint32_t w = 0;
    if (g + 4 <= total) {
      w = *reinterpret_cast<const uint32_t *>(a.bytes + g);
    } else {
      for (uint32_t t = 0; t < 4; ++t)
        if (g + t < total) w |= static_cast<uint32_t>(a.bytes[g + t]) << (8 * t);
    }
    lds[k] = w;
  }
  return al;
}

// WPE: amdgpu_waves_per_eu hint (VGPR budget); the kernels are bound by the
// latency of dependent trie loads, so occupancy matters more than spills.
template <int W, int WPE>
__global__ __launch_bounds__(kEBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void estep_forward_kernel(EArgs a) {
  constexpr int kEAmb = kAmbEntries;
  __shared__ uint32_t lds_bp[(kELdsBp / 4) * kEBlock];
  uint8_t *lbp = reinterpret_cast<uint8_t *>(lds_bp);
  const int tid = threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kEBlock;
  __shared__ uint32_t lds_stage[kEStage / 4];
  const uint8_t *lsb = reinterpret_cast<const uint8_t *>(lds_stage);
  const uint64_t total_bytes = a.off[a.n];
  __shared__ uint32_t lds_sort[2 * kEBlock];
  // (unit, score) of the root's children: every walk's first trie step from
  // LDS (as in the encode byte kernel); the first SortedLane barrier covers it.
  __shared__ uint2 lds_root[kEBlock];
  {
    const uint32_t nd = a.root_base ^ static_cast<uint32_t>(tid);
    lds_root[tid] = nd < a.num_units ? a.uvs[nd] : make_uint2(0u, 0u);
  }
  for (uint64_t blk = static_cast<uint64_t>(blockIdx.x) * kEBlock; blk < a.n; blk += stride) {
    const uint64_t al = StageBlockBytes(a, blk, lds_stage, total_bytes);
    const uint64_t i = blk + SortedLane(a, blk, lds_sort);  // (its barriers cover the staging)
    [&]() {
    if (i >= a.n) return;
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    if (nb == 0) {
      a.Zlat[i] = 0.f;
      a.N[i] = 0;
      a.ntok[i] = 0;
      return;
    }
    const uint64_t lso = b0 - al;
    // Bytes past the LDS stage come through a buffer resource from the
    // block's aligned start: a separate intrinsic keeps the compiler from
    // merging the two branches into flat loads (which pay the global path's
    // latency and counters for LDS hits too).  A sentence reaching past the
    // resource's 2 GB range is flagged below (general kernel).
    const uint64_t brem = total_bytes - al;
    const uint32_t bnrec = static_cast<uint32_t>(brem < 0x7FFFFFF0ull ? brem : 0x7FFFFFF0ull);
    const auto brsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.bytes + al), 0, static_cast<int>(bnrec), 0x00020000);
    auto sb = [&](uint32_t x) -> uint32_t {
      const uint32_t pp = static_cast<uint32_t>(lso) + x;
      return pp < kEStage ? static_cast<uint32_t>(lsb[pp])
                          : static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b8(brsrc, pp, 0, 0));
    };
    float *__restrict__ Ab = a.A + b0;
    // Back-pointers past the LDS window: a buffer resource over the scratch
    // (total_bytes + 1 bytes from offset 0; position nb of the last sentence
    // included), addressed like the bytes.
    const uint64_t bprem = total_bytes + 1 - al;
    const auto bprsrc = __builtin_amdgcn_make_buffer_rsrc(
        a.gbp + al, 0, static_cast<int>(bprem < 0x7FFFFFFFull ? bprem : 0x7FFFFFFFull), 0x00020000);
    auto bp_store = [&](uint32_t pos, uint32_t v) {
      if (pos < kELdsBp) lbp[((pos >> 2) * kEBlock + tid) * 4 + (pos & 3)] = static_cast<uint8_t>(v);
      else __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), bprsrc, static_cast<uint32_t>(lso) + pos, 0, 0);
    };
    auto bp_load = [&](uint32_t pos) -> uint32_t {
      return pos < kELdsBp ? lbp[((pos >> 2) * kEBlock + tid) * 4 + (pos & 3)]
                           : __builtin_amdgcn_raw_buffer_load_b8(bprsrc, static_cast<uint32_t>(lso) + pos, 0, 0);
    };
    float T[W], Ar[W];
    uint32_t B[W];  // slot d's running-max setter (begin byte offset)
#pragma unroll
    for (int d = 0; d < W; ++d) {
      T[d] = 0.f;
      Ar[d] = 0.f;
      B[d] = 0;
    }
    uint64_t has = 1;
    uint32_t ae[kEAmb], aB2[kEAmb];
    float aT[kEAmb], aT2[kEAmb];
#pragma unroll
    for (int k = 0; k < kEAmb; ++k) {
      ae[k] = kNone;
      aB2[k] = 0;
      aT[k] = 0.f;
      aT2[k] = 0.f;
    }
    bool bad = lso + nb > bnrec, any_amb = false;
    uint32_t nodes = 0;
    // end_of(): byte offset of the node's end, derived only on the (rare)
    // running-max path from the char-end mask of the current walk.
    auto insert = [&](auto dc, float s_node, float A_p, float T0, uint32_t begin, auto end_of) {
      constexpr int d = decltype(dc)::value;
      const float bt = __fadd_rn(T0, s_node);
      const bool first = !((has >> d) & 1);
      Ar[d] = LogSumExpDev(Ar[d], __fadd_rn(s_node, A_p), first);
      if (first) {
        has |= (1ull << d);
        T[d] = bt;
        B[d] = begin;
      } else if (bt > T[d]) {
        const uint32_t end = end_of();
        const bool nr = NearTie(T[d], bt, a.tie_mag);
        int slot = -1, free_slot = -1;
#pragma unroll
        for (int k = 0; k < kEAmb; ++k) {
          if (ae[k] == end) slot = k;
          if (ae[k] == kNone && free_slot < 0) free_slot = k;
        }
        if (slot >= 0) {
#pragma unroll
          for (int k = 0; k < kEAmb; ++k)
            if (k == slot) {
              if (NearTie(aT2[k], bt, a.tie_mag)) bad = true;
              if (nr) {
                aT2[k] = T[d];
                aB2[k] = B[d];
                aT[k] = bt;
              } else {
                ae[k] = kNone;
              }
            }
        } else if (nr) {
          if (free_slot < 0) bad = true;
          any_amb = true;
#pragma unroll
          for (int k = 0; k < kEAmb; ++k)
            if (k == free_slot) {
              ae[k] = end;
              aT2[k] = T[d];
              aB2[k] = B[d];
              aT[k] = bt;
            }
        }
        T[d] = bt;
        B[d] = begin;
      }
    };
    uint32_t pos = 0;
    for (;;) {
      if (pos > 0) bp_store(pos, pos - B[0]);
      const float A_p = Ar[0];
      if (pos >= nb) break;
      Ab[pos] = A_p;
      const float T0 = T[0];
      uint32_t base_u = a.root_base, q = pos, clen0 = 1;
      bool alive = true, single = false;
      // Phase 1: the walk; each step's (unit, score) gather also gives a
      // leaf's score.
      uint32_t lnode[W];  // leaf score bits
      uint32_t leaf = 0;
      uint64_t cend = 0;  // bit k: a char ends k + 1 bytes after pos
      auto stepd = [&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if (alive) {
          if (q >= nb) {
            alive = false;
          } else {
            const uint32_t lead = sb(q);
            uint32_t cl = OneCharLenDev(lead);
            if (cl > nb - q) cl = nb - q;
            if (d == 1) clen0 = cl;
            // Structure check for the backward pass: a char start must not
            // be a continuation byte, and its tail must be continuation bytes.
            if (d == 1) {
              if (ContinuationByte(lead)) bad = true;
              for (uint32_t j = 1; j < cl; ++j)
                if (!ContinuationByte(sb(q + j))) bad = true;
            }
            uint32_t u = 0, sc = 0;
            for (uint32_t j = 0; j < cl; ++j) {
              const uint32_t c = j == 0 ? lead : sb(q + j);
              const uint2 x = (d == 1 && j == 0) ? lds_root[c] : c ? a.uvs[base_u ^ c] : make_uint2(0u, 0u);
              u = x.x;
              sc = x.y;
              if ((u & 0xFFu) != c || c == 0) {
                alive = false;
                break;
              }
              base_u = u >> 9;
              if (j + 1 < cl && (u & 0x100u)) {  // leaf inside a char: general path
                bad = true;
                ++nodes;
                if (d == 1) single = true;
              }
            }
            if (alive) {
              q += cl;
              // The char-end mask covers 64 bytes; a longer walk (W = 32 with
              // multi-byte chars) goes to the general kernel.
              if (q - pos > 64) bad = true;
              else cend |= 1ull << (q - pos - 1);
              if (u & 0x100u) {
                lnode[d] = sc;
                leaf |= 1u << d;
                ++nodes;
                if (d == 1) single = true;
              }
            }
          }
        }
      };
      StaticFor<1, W>(stepd);
      // Phase 3: inserts in ascending length (then UNK at length 1).
      StaticFor<1, W>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if ((leaf >> d) & 1)
          insert(dc, __uint_as_float(lnode[d]), A_p, T0, pos, [&]() -> uint32_t {
            uint64_t m = cend;
            for (int k = 1; k < d; ++k) m &= m - 1;  // drop the first d-1 char ends
            return pos + static_cast<uint32_t>(__builtin_ctzll(m)) + 1;
          });
        if (d == 1 && !single) {  // UNK node, id = unk_id_ = 0 (TrainerModel)
          insert(dc, a.unk_score, A_p, T0, pos, [&]() -> uint32_t { return pos + clen0; });
          ++nodes;
        }
      });
#pragma unroll
      for (int d = 0; d + 1 < W; ++d) {
        T[d] = T[d + 1];
        Ar[d] = Ar[d + 1];
        B[d] = B[d + 1];
      }
      T[W - 1] = 0.f;
      Ar[W - 1] = 0.f;
      B[W - 1] = 0;
      has >>= 1;
      pos += clen0;
    }
    const float Z = Ar[0];  // alpha[EOS]
    a.Zlat[i] = Z;
    a.N[i] = nodes;
    auto flag = [&]() {
      a.ntok[i] = kNone;
      const uint32_t k = atomicAdd(&a.status[0], 1u);
      a.flagged[k] = static_cast<uint32_t>(i);
      atomicMax(&a.status[1], nb);
    };
    if (bad) {
      flag();
      return;
    }
    // Viterbi().size(): backtrace count (node scores only to resolve ties).
    // Every step must move left (begin < end): an inconsistent back-pointer
    // sends the sentence to the general kernel instead of looping.
    uint32_t e = nb, k = 0;
    float rs = 0.f;
    while (e > 0) {
      uint32_t b = e - bp_load(e);
#pragma unroll
      for (int t = 0; t < kEAmb; ++t)
        if (ae[t] == e && __fadd_rn(aT2[t], rs) == __fadd_rn(aT[t], rs)) b = aB2[t];
      if (b >= e || k >= nb) {
        flag();
        return;
      }
      if (any_amb) {
        uint32_t nbase = a.root_base, node = 0, u = 0;
        bool found = true;
        for (uint32_t j = b; j < e; ++j) {
          const uint32_t c = sb(j);
          node = nbase ^ c;
          u = c ? a.units[node] : 0u;
          if ((u & 0xFFu) != c || c == 0) {
            found = false;
            break;
          }
          nbase = u >> 9;
        }
        rs = (found && (u & 0x100u)) ? a.scores[a.values[node]] : a.unk_score;
      }
      ++k;
      e = b;
    }
    a.ntok[i] = k;
      }();
    __syncthreads();
  }
}

// kVar bit 0: lagged emits — node d's id/score loads are issued right after
// walk step d and the node is emitted at step d + 1 (its loads have landed by
// then), so the 2 x 16 id/score registers of the batched version are not live
// across the walk.  PARITY records of a position are then written from the
// block's end backwards: a position's trie nodes have distinct piece ids, so
// their relative order does not matter to the per-key fold; the UNK record
// (id 0, which can equal a multi-char trie piece's id 0) gets the block's last
// slot, reserved once step 1 has decided it, so it still follows every trie
// node as in begin_nodes order.  Bit 1: PARITY-only build without the FAST
// LDS accumulators (47 -> 15 KB of LDS per block).
template <int W, int WPE, int kVar = 0>
__global__ __launch_bounds__(kEBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void estep_backward_kernel(EArgs a) {
  constexpr bool kLag = (kVar & 1) != 0;
  constexpr bool kParityOnly = (kVar & 2) != 0;
  // kPair: two char positions per lane in flight (kLag is ignored): the
  // walks of position q and of the char start before it issue their trie
  // gathers together, then both positions' nodes are emitted in descending
  // position order (the emission needs q's Bt before the earlier one's).
  constexpr bool kPair = (kVar & 4) != 0;
  // kRoll: a position's nodes are emitted by a loop over the lane's own
  // present nodes (a wave runs it max-over-lanes times) instead of one
  // predicated emission per ring depth (a wave pays every depth any lane has
  // a node at: the union).  The loop body selects the node's registers.
  constexpr bool kRoll = (kVar & 8) != 0;
  // kStage (with kRoll and kParityOnly, deferred records): a lane's kept
  // records go to an LDS ring of kRecStage entries and are written to their
  // slots as one contiguous run per flush.  Written one by one, the 4-byte
  // key / ex stores of 64 lanes hit 64 scattered lines per instruction: L2
  // evicted half-written lines (write traffic) and filled them for the
  // partial writes (read traffic), and the walk's trie lines went with them.
  constexpr bool kStage = (kVar & 16) != 0 && kRoll && kParityOnly;
  // kAT (with kRoll): the byte-kernel forward pass's tile-transposed alpha
  // and lane assignment (EArgs::AT, lanemap), and with kParityOnly the
  // tile-transposed deferred records (EArgs::RT).
  constexpr bool kAT = (kVar & 32) != 0 && kRoll;
  constexpr uint32_t kRecStage = 8;
  __shared__ uint32_t lds_rk[kStage ? kRecStage * kEBlock : 1];
  __shared__ float lds_rx[kStage ? kRecStage * kEBlock : 1];
  // FAST: the expected counts of the kHot highest-score (= most frequent)
  // pieces are privatised per block in LDS and flushed once, so the hot ids
  // ("▁", single letters) do not serialise on global fp64 atomics.
  __shared__ double lds_acc[kParityOnly ? 1 : kHot];
  if (!kParityOnly && a.mode == SPM_ESTEP_FAST) {
    for (int s = threadIdx.x; s < kHot; s += kEBlock) lds_acc[s] = 0.0;
    __syncthreads();
  }
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kEBlock;
  double obj_local = 0.0;
  int64_t ntok_local = 0;
  __shared__ uint32_t lds_stage[kEStage / 4];
  const uint8_t *lsb = reinterpret_cast<const uint8_t *>(lds_stage);
  const uint64_t total_bytes = a.off[a.n];
  __shared__ uint32_t lds_sort[2 * kEBlock];
  __shared__ uint4 lds_root[kEBlock];  // root children (unit, id, score, hot slot + 1)
  {
    const uint32_t nd = a.root_base ^ static_cast<uint32_t>(threadIdx.x);
    lds_root[threadIdx.x] = nd < a.num_units ? a.uvis[nd] : make_uint4(0u, 0u, 0u, 0u);
  }
  // PARITY record drop: a record c >= 0 that is below a quarter ulp of a
  // lower bound of its float accumulator cannot change it (see
  // estep_threshold_kernel); the bound's exponent per hot piece sits in LDS
  // and is packed into the node's id register (ids < 2^24) at the walk step.
  __shared__ uint8_t lds_drop[kParityOnly ? kHot : 4];
  const bool drop = kParityOnly && a.drop_exp != nullptr;
  if (drop) {
    for (int s = threadIdx.x; s < kHot / 4; s += kEBlock)
      reinterpret_cast<uint32_t *>(lds_drop)[s] = reinterpret_cast<const uint32_t *>(a.drop_exp)[s];
  }
  for (uint64_t blk = static_cast<uint64_t>(blockIdx.x) * kEBlock; blk < a.n; blk += stride) {
    const uint64_t al = StageBlockBytes(a, blk, lds_stage, total_bytes);
    uint64_t i;
    if constexpr (kAT) {  // the forward pass's lane assignment
      __syncthreads();  // (covers the staging)
      i = blk + a.lanemap[blk + threadIdx.x];
    } else {
      i = blk + SortedLane(a, blk, lds_sort);  // (its barriers cover the staging)
    }
    // The tile's AT / RT blocks (uniform; a lane adds its column).
    const float *__restrict__ ATt = kAT ? a.AT + (blk >> 8) * (kATRows * kEBlock) : nullptr;
    uint2 *__restrict__ RTt = kAT && kParityOnly && a.RT ? a.RT + (blk >> 8) * (kRTRows * kEBlock) : nullptr;
    [&]() {
    if (i >= a.n) return;
    const uint32_t nt = a.ntok[i];
    if (nt == kNone) {  // general path (its records go to the range slots)
      if (kAT && kParityOnly && RTt) a.colmap[i] = 0xFFFFu;
      return;
    }
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    const float freq_f = static_cast<float>(a.freq[i]);
    const float lfreq = a.exs ? logf(freq_f) : 0.f;  // deferred records' drop test
    const float Z = a.Zlat[i];
    const uint32_t bucket = a.mode == SPM_ESTEP_PARITY ? BucketOf(a, i) : 0;
    if (a.mode == SPM_ESTEP_FAST) {
      // obj -= (freq * Z) / all_sentence_freq  (float ops, summed in fp64)
      obj_local -= static_cast<double>(__fdiv_rn(__fmul_rn(freq_f, Z), a.all_freq_f));
      ntok_local += nt;
    }
    if (nb == 0) return;
    const uint64_t lso = b0 - al;
    // As in the forward kernel (which flagged any sentence past the range).
    const uint64_t brem = total_bytes - al;
    const auto brsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.bytes + al), 0, static_cast<int>(brem < 0x7FFFFFF0ull ? brem : 0x7FFFFFF0ull),
        0x00020000);
    auto sb = [&](uint32_t x) -> uint32_t {
      const uint32_t pp = static_cast<uint32_t>(lso) + x;
      return pp < kEStage ? static_cast<uint32_t>(lsb[pp])
                          : static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b8(brsrc, pp, 0, 0));
    };
    const float *__restrict__ Ab = a.A + b0;
    auto alpha = [&](uint32_t q) -> float {
      if constexpr (kAT)
        if (q < kATRows) return ATt[q * kEBlock + threadIdx.x];
      return Ab[q];
    };
    float Br[W];
#pragma unroll
    for (int d = 0; d < W; ++d) Br[d] = 0.f;  // Br[1] = Bt[len] = 0 (EOS)
    uint64_t cursor = a.mode == SPM_ESTEP_PARITY ? a.rec_off[i] + a.N[i] : 0;
    uint32_t rt_k = 0;  // RT: records this lane kept so far
    // kStage: records staged in LDS (entry k of nst belongs at slot
    // w + nst - 1 - k, w = the lane's cursor); written in ascending order.
    uint32_t nst = 0;
    auto stage_flush = [&](uint64_t wc) {
      if constexpr (kStage) {
        for (uint32_t k = nst; k-- > 0;) {
          const uint64_t g = wc + nst - 1 - k;
          a.keys[g] = lds_rk[k * kEBlock + threadIdx.x];
          a.exs[g] = lds_rx[k * kEBlock + threadIdx.x];
        }
        nst = 0;
      }
    };
    // Last char start.
    uint32_t q = nb - 1;
    while (q > 0 && ContinuationByte(sb(q))) --q;
    if constexpr (kPair) {
      const bool parity = kParityOnly || a.mode == SPM_ESTEP_PARITY;
      uint64_t w = cursor;  // PARITY records, written from the range's end down
      // One node's record or FAST accumulation (c = freq * exp(...),
      // :318-325); PARITY-only drop test as in the lagged kernel.
      auto record = [&](float A_q, int32_t packed, float sc, float be) {
        const float ex = __fsub_rn(__fadd_rn(__fadd_rn(A_q, sc), be), Z);
        const uint32_t id = kParityOnly ? static_cast<uint32_t>(packed) & 0xFFFFFFu : static_cast<uint32_t>(packed);
        if (parity) {
          ParityRecord(a, w, bucket * a.V + id, ex, freq_f, lfreq, kParityOnly ? static_cast<uint32_t>(packed) >> 24 : 0u);
        } else if constexpr (!kParityOnly) {
          const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
          const int32_t hs = a.hot_slot[id];
          if (hs >= 0) atomicAdd(&lds_acc[hs], c);
          else atomicAdd(&a.acc[id], c);
        }
      };
      // Position q's begin_nodes: records (UNK first: it must sit above the
      // trie nodes' records, piece 0 may be among them), LogSumExp terms in
      // the reference order (trie nodes by length, then UNK), Bt[q] into the
      // ring.  Records of one position have distinct keys but UNK's, so
      // their order inside the position is free.
      auto emit_pos = [&](float A_q, const float (&sd)[W], const int32_t (&id)[W], uint64_t pres, bool single) {
        const bool unk = !single;
        if (unk) record(A_q, 0, a.unk_score, Br[1]);
        float bt = 0.f;
        bool first = true;
        StaticFor<1, W>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if ((pres >> d) & 1) {
            record(A_q, id[d], sd[d], Br[d]);
            bt = LogSumExpDev(bt, __fadd_rn(sd[d], Br[d]), first);
            first = false;
          }
        });
        if (unk) bt = LogSumExpDev(bt, __fadd_rn(a.unk_score, Br[1]), first);
#pragma unroll
        for (int d = W - 1; d >= 2; --d) Br[d] = Br[d - 1];
        Br[1] = bt;
      };
      const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
      uint32_t qa = q;
      for (;;) {
        const bool hb = qa > 0;
        uint32_t qb = 0;
        if (hb) {
          qb = qa - 1;
          while (qb > 0 && ContinuationByte(sb(qb))) --qb;
        }
        const float A_a = alpha(qa);
        const float A_b = hb ? alpha(qb) : 0.f;
        uint32_t ba = a.root_base, bb = a.root_base, pa = qa, pb = qb;
        bool la = true, lb = hb, one_a = false, one_b = false;
        float sda[W], sdb[W];
        int32_t ida[W], idb[W];
        uint64_t pra = 0, prb = 0;
        // A chain's char step after its first gather landed: the char's
        // remaining bytes (multi-byte chars only) and the node, if a leaf.
        auto finish = [&](auto dc, bool &l, uint32_t &base, uint32_t &p, uint32_t c, uint32_t cl, uint4 x,
                          float (&sd)[W], int32_t (&id)[W], uint64_t &pres, bool &one) {
          constexpr int d = decltype(dc)::value;
          if (!l) return;
          if ((x.x & 0xFFu) != c || c == 0) {
            l = false;
            return;
          }
          base = x.x >> 9;
          for (uint32_t j = 1; j < cl; ++j) {
            const uint32_t cj = sb(p + j);
            x = cj ? a.uvis[base ^ cj] : z4;
            if ((x.x & 0xFFu) != cj || cj == 0) {
              l = false;
              return;
            }
            base = x.x >> 9;
          }
          p += cl;
          if (x.x & 0x100u) {
            id[d] = static_cast<int32_t>(x.y);
            if constexpr (kParityOnly)
              if (drop && x.w) id[d] |= static_cast<int32_t>(static_cast<uint32_t>(lds_drop[x.w - 1]) << 24);
            sd[d] = __uint_as_float(x.z);
            pres |= 1ull << d;
            if (d == 1) one = true;
          }
        };
        StaticFor<1, W>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          sda[d] = 0.f;
          sdb[d] = 0.f;
          ida[d] = 0;
          idb[d] = 0;
          // Issue both chains' first-byte gathers, then complete each.
          uint32_t ca = 0, cb = 0, cla = 0, clb = 0;
          uint4 xa = z4, xb = z4;
          if (la) {
            if (pa >= nb) {
              la = false;
            } else {
              ca = sb(pa);
              cla = OneCharLenDev(ca);
              if (cla > nb - pa) cla = nb - pa;
              xa = d == 1 ? lds_root[ca] : ca ? a.uvis[ba ^ ca] : z4;
            }
          }
          if (lb) {
            if (pb >= nb) {
              lb = false;
            } else {
              cb = sb(pb);
              clb = OneCharLenDev(cb);
              if (clb > nb - pb) clb = nb - pb;
              xb = d == 1 ? lds_root[cb] : cb ? a.uvis[bb ^ cb] : z4;
            }
          }
          finish(dc, la, ba, pa, ca, cla, xa, sda, ida, pra, one_a);
          finish(dc, lb, bb, pb, cb, clb, xb, sdb, idb, prb, one_b);
        });
        emit_pos(A_a, sda, ida, pra, one_a);
        if (!hb) break;
        emit_pos(A_b, sdb, idb, prb, one_b);
        if (qb == 0) break;
        qa = qb - 1;
        while (qa > 0 && ContinuationByte(sb(qa))) --qa;
      }
      if (parity) cursor = w;
    } else
    for (;;) {
      const float A_q = alpha(q);
      uint32_t base_u = a.root_base, p = q;
      bool alive = true, single = false;
      float sd[W];
      int32_t idd[W];
      uint64_t present = 0;
      auto stepd = [&](auto dc) {
        constexpr int d = decltype(dc)::value;
        sd[d] = 0.f;
        idd[d] = 0;
        if (alive) {
          if (p >= nb) {
            alive = false;
          } else {
            const uint32_t lead = sb(p);
            uint32_t cl = OneCharLenDev(lead);
            if (cl > nb - p) cl = nb - p;
            uint4 x = make_uint4(0u, 0u, 0u, 0u);
            for (uint32_t j = 0; j < cl; ++j) {
              const uint32_t c = j == 0 ? lead : sb(p + j);
              x = (d == 1 && j == 0) ? lds_root[c] : c ? a.uvis[base_u ^ c] : make_uint4(0u, 0u, 0u, 0u);
              if ((x.x & 0xFFu) != c || c == 0) {
                alive = false;
                break;
              }
              base_u = x.x >> 9;
            }
            if (alive) {
              p += cl;
              if (x.x & 0x100u) {
                idd[d] = static_cast<int32_t>(x.y);
                if constexpr (kParityOnly)
                  if (drop && x.w) idd[d] |= static_cast<int32_t>(static_cast<uint32_t>(lds_drop[x.w - 1]) << 24);
                sd[d] = __uint_as_float(x.z);
                present |= 1ull << d;
                if (d == 1) single = true;
              }
            }
          }
        }
      };
      if constexpr (kLag) {
        const bool parity = kParityOnly || a.mode == SPM_ESTEP_PARITY;
        uint64_t w = cursor;  // records written from the sentence range's end down
        float bt = 0.f;
        bool first = true, unk = false;
        // One node's record (c = freq * exp(...), :318-325); kept unless the
        // drop test proves it cannot change its accumulator.  Packed ids carry
        // the accumulator bound's biased float exponent in bits 24-31.
        auto record = [&](int32_t packed, float sc, float be) {
          const float ex = __fsub_rn(__fadd_rn(__fadd_rn(A_q, sc), be), Z);
          const uint32_t id = kParityOnly ? static_cast<uint32_t>(packed) & 0xFFFFFFu : static_cast<uint32_t>(packed);
          if (parity) {
            // c < 2^(e_exp - 152) = ulp(bound) / 4 is a no-op (ParityRecord).
            ParityRecord(a, w, bucket * a.V + id, ex, freq_f, lfreq,
                         kParityOnly ? static_cast<uint32_t>(packed) >> 24 : 0u);
          } else if constexpr (!kParityOnly) {
            const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
            const int32_t hs = a.hot_slot[id];
            if (hs >= 0) atomicAdd(&lds_acc[hs], c);
            else atomicAdd(&a.acc[id], c);
          }
        };
        auto lse = [&](float sc, float be) {
          bt = LogSumExpDev(bt, __fadd_rn(sc, be), first);
          first = false;
        };
        // The UNK node of begin_nodes[q] comes after the trie nodes in the
        // reference order (its LogSumExp term is applied last), but its record
        // is written first: records go downwards, so it ends up above the
        // trie nodes' ones (piece 0, also the TrainerModel's UNK id, may be
        // among them and its record must precede).
        // (UNK records carry no bound and are always kept.)
        StaticFor<1, W + 1>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if constexpr (d < W) {
            stepd(dc);
            if constexpr (d == 1) {
              unk = !single;
              if (unk) record(0, a.unk_score, Br[1]);
            }
          }
          if constexpr (d >= 2) {
            if ((present >> (d - 1)) & 1) {
              record(idd[d - 1], sd[d - 1], Br[d - 1]);
              lse(sd[d - 1], Br[d - 1]);
            }
          }
        });
        if (unk) lse(a.unk_score, Br[1]);
        if (parity) cursor = w;
#pragma unroll
        for (int d = W - 1; d >= 2; --d) Br[d] = Br[d - 1];
        Br[1] = bt;
        if (q == 0) break;
        --q;
        while (q > 0 && ContinuationByte(sb(q))) --q;
        continue;
      }
      StaticFor<1, W>(stepd);
      if constexpr (kRoll) {
        const bool parity = kParityOnly || a.mode == SPM_ESTEP_PARITY;
        uint64_t w = cursor;  // PARITY records, written from the range's end down
        auto rec = [&](int32_t packed, float sc, float be) {
          const float ex = __fsub_rn(__fadd_rn(__fadd_rn(A_q, sc), be), Z);
          const uint32_t id = kParityOnly ? static_cast<uint32_t>(packed) & 0xFFFFFFu : static_cast<uint32_t>(packed);
          if constexpr (kStage) {
            if (a.exs) {
              if (!DeferredKeep(ex, freq_f, lfreq, static_cast<uint32_t>(packed) >> 24)) return;
              --w;
              lds_rk[nst * kEBlock + threadIdx.x] = bucket * a.V + id;
              lds_rx[nst * kEBlock + threadIdx.x] = ex;
              if (++nst == kRecStage) stage_flush(w);
              return;
            }
          }
          if (parity) {
            if (kAT && kParityOnly && RTt) {  // deferred records, tile-transposed
              if (!DeferredKeep(ex, freq_f, lfreq, static_cast<uint32_t>(packed) >> 24)) return;
              --w;
              const uint32_t k = rt_k++;
              if (k < kRTRows) RTt[k * kEBlock + threadIdx.x] = make_uint2(bucket * a.V + id, __float_as_uint(ex));
              else StoreRecordEx(a, w, bucket * a.V + id, ex);
              return;
            }
            ParityRecord(a, w, bucket * a.V + id, ex, freq_f, lfreq,
                         kParityOnly ? static_cast<uint32_t>(packed) >> 24 : 0u);
          } else if constexpr (!kParityOnly) {
            const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
            const int32_t hs = a.hot_slot[id];
            if (hs >= 0) atomicAdd(&lds_acc[hs], c);
            else atomicAdd(&a.acc[id], c);
          }
        };
        // UNK's record first (above the trie nodes' ones, as the lagged
        // kernel), its LogSumExp term last (begin_nodes order).
        const bool unk = !single;
        if (unk) rec(0, a.unk_score, Br[1]);
        float bt = 0.f;
        bool first = true;
        uint32_t m = static_cast<uint32_t>(present);
        while (m) {
          const uint32_t d = static_cast<uint32_t>(__builtin_ctz(m));  // ascending length
          m &= m - 1;
          float sc = sd[1], be = Br[1];
          int32_t id = idd[1];
          StaticFor<2, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if (d == static_cast<uint32_t>(k)) {
              sc = sd[k];
              be = Br[k];
              id = idd[k];
            }
          });
          rec(id, sc, be);
          bt = LogSumExpDev(bt, __fadd_rn(sc, be), first);
          first = false;
        }
        if (unk) bt = LogSumExpDev(bt, __fadd_rn(a.unk_score, Br[1]), first);
        if (parity) cursor = w;
#pragma unroll
        for (int d = W - 1; d >= 2; --d) Br[d] = Br[d - 1];
        Br[1] = bt;
        if (q == 0) break;
        --q;
        while (q > 0 && ContinuationByte(sb(q))) --q;
        continue;
      }
      // begin_nodes[q] order: trie nodes by ascending length, then UNK.
      const bool unk = !single;
      const uint32_t g = __popcll(present) + (unk ? 1u : 0u);
      if (a.mode == SPM_ESTEP_PARITY) cursor -= g;
      uint64_t w = cursor;
      float bt = 0.f;
      bool first = true;
      auto emit = [&](int32_t id, float sc, float be) {
        const float ex = __fsub_rn(__fadd_rn(__fadd_rn(A_q, sc), be), Z);
        if (a.mode == SPM_ESTEP_PARITY) {
          const uint32_t key = bucket * a.V + static_cast<uint32_t>(id);
          if (a.exs) StoreRecordEx(a, w, key, ex);
          else StoreRecord(a, w, key, static_cast<double>(freq_f) * exp(static_cast<double>(ex)));
          ++w;
        } else {
          const double c = static_cast<double>(freq_f) * exp(static_cast<double>(ex));
          if constexpr (!kParityOnly) {
            const int32_t hs = a.hot_slot[id];
            if (hs >= 0) atomicAdd(&lds_acc[hs], c);
            else atomicAdd(&a.acc[id], c);
          }
        }
        bt = LogSumExpDev(bt, __fadd_rn(sc, be), first);
        first = false;
      };
      auto emitd = [&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if ((present >> d) & 1) emit(idd[d], sd[d], Br[d]);
      };
      StaticFor<1, W>(emitd);
      if (unk) emit(0, a.unk_score, Br[1]);
      // Shift: slot d+1 <- d; slot 1 = Bt[q].
#pragma unroll
      for (int d = W - 1; d >= 2; --d) Br[d] = Br[d - 1];
      Br[1] = bt;
      if (q == 0) break;
      --q;
      while (q > 0 && ContinuationByte(sb(q))) --q;
    }
    if constexpr (kStage)
      if (nst) stage_flush(cursor);
    // Records kept: the last `kept` slots of the sentence's range.
    if (kParityOnly && drop) a.kept[i] = static_cast<uint32_t>(a.rec_off[i] + a.N[i] - cursor);
      }();
    __syncthreads();
  }
  if (!kParityOnly && a.mode == SPM_ESTEP_FAST) {
    __syncthreads();
    for (int s = threadIdx.x; s < kHot; s += kEBlock)
      if (lds_acc[s] != 0.0) atomicAdd(&a.acc[a.hot_id[s]], lds_acc[s]);
    // wave reduce, one atomic per wave
    for (int o = 32; o >= 1; o >>= 1) {
      obj_local += __shfl_xor(obj_local, o);
      ntok_local += __shfl_xor(ntok_local, o);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(a.acc_obj, obj_local);
      atomicAdd(reinterpret_cast<unsigned long long *>(a.ntok_b),
                static_cast<unsigned long long>(ntok_local));
    }
  }
}

// ---------------------------------------------------------------------------
// General kernel: the reference lattice literally (TrainerModel semantics:
// unk_id 0, every piece NORMAL), one flagged sentence per lane.
// ---------------------------------------------------------------------------
struct EGenArgs {
  EArgs a;
  const uint32_t *__restrict__ list;
  const uint32_t *__restrict__ count;
  uint8_t *__restrict__ scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;
  int K;
  uint32_t *__restrict__ error;
};

__global__ __launch_bounds__(64) void estep_general_kernel(EGenArgs g) {
  const EArgs &a = g.a;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t total = *g.count;
  for (uint64_t j = tid; j < total; j += nthreads) {
    const uint32_t i = g.list[j];
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    if (nb > g.max_nb) {
      atomicOr(g.error, 1u);
      continue;
    }
    const uint8_t *__restrict__ s = a.bytes + b0;
    uint8_t *slab = g.scratch + tid * g.slab_bytes;
    const uint32_t cap = nb * g.K + 2;
    uint32_t *cs = reinterpret_cast<uint32_t *>(slab);
    int32_t *end_head = reinterpret_cast<int32_t *>(cs + nb + 1);
    int32_t *end_tail = end_head + nb + 1;
    int32_t *bfirst = end_tail + nb + 1;
    int32_t *bcount = bfirst + nb + 1;
    float *nscore = reinterpret_cast<float *>(bcount + nb + 1);
    float *nbt = nscore + cap;
    float *nal = nbt + cap;
    float *nbe = nal + cap;
    int32_t *nid = reinterpret_cast<int32_t *>(nbe + cap);
    int32_t *nprev = nid + cap;
    int32_t *nnext = nprev + cap;
    uint32_t *npos = reinterpret_cast<uint32_t *>(nnext + cap);
    uint32_t *nlen = npos + cap;
    uint32_t nc = 0;
    for (uint32_t q = 0; q < nb;) {
      cs[nc++] = q;
      const uint32_t cl = OneCharLenDev(s[q]);
      q += cl < nb - q ? cl : nb - q;
    }
    cs[nc] = nb;
    for (uint32_t p = 0; p <= nc; ++p) {
      end_head[p] = end_tail[p] = -1;
      bfirst[p] = bcount[p] = 0;
    }
    auto push_end = [&](uint32_t q, int32_t nd) {
      nnext[nd] = -1;
      if (end_tail[q] < 0) end_head[q] = nd;
      else nnext[end_tail[q]] = nd;
      end_tail[q] = nd;
    };
    auto init_node = [&](int32_t nd, uint32_t p, uint32_t len, int32_t id, float sc) {
      nscore[nd] = sc;
      nbt[nd] = 0.f;
      nal[nd] = 0.f;
      nbe[nd] = 0.f;
      nid[nd] = id;
      nprev[nd] = -1;
      npos[nd] = p;
      nlen[nd] = len;
    };
    init_node(0, 0, 0, -1, 0.f);  // BOS
    push_end(0, 0);
    init_node(1, nc, 0, -1, 0.f);  // EOS
    int32_t nn = 2;
    bfirst[nc] = 1;
    bcount[nc] = 1;
    for (uint32_t p = 0; p < nc; ++p) {
      bfirst[p] = nn;
      bool single = false;
      uint32_t base = a.root_base, cpos = p;
      for (uint32_t q = cs[p]; q < nb; ++q) {
        const uint32_t c = s[q];
        if (c == 0) break;
        const uint32_t node = base ^ c;
        const uint32_t u = a.units[node];
        if ((u & 0xFFu) != c) break;
        base = u >> 9;
        if (u & 0x100u) {
          while (cs[cpos] < q + 1) ++cpos;
          const uint32_t length = cpos - p;
          const int32_t id = a.values[node];
          const int32_t nd = nn++;
          init_node(nd, p, length, id, a.scores[id]);
          push_end(p + length, nd);
          if (length == 1) single = true;
        }
      }
      if (!single) {
        const int32_t nd = nn++;
        init_node(nd, p, 1, 0, a.unk_score);
        push_end(p + 1, nd);
      }
      bcount[p] = nn - bfirst[p];
    }
    auto begin_list = [&](uint32_t p, int32_t k) -> int32_t { return bfirst[p] + k; };
    // PopulateMarginal (unigram_model.cc:272-328)
    for (uint32_t p = 0; p <= nc; ++p)
      for (int32_t k = 0; k < bcount[p]; ++k) {
        const int32_t r = begin_list(p, k);
        for (int32_t l = end_head[p]; l >= 0; l = nnext[l])
          nal[r] = LogSumExpDev(nal[r], __fadd_rn(nscore[l], nal[l]), l == end_head[p]);
      }
    for (int64_t p = nc; p >= 0; --p)
      for (int32_t l = end_head[p]; l >= 0; l = nnext[l])
        for (int32_t k = 0; k < bcount[p]; ++k) {
          const int32_t r = begin_list(static_cast<uint32_t>(p), k);
          nbe[l] = LogSumExpDev(nbe[l], __fadd_rn(nscore[r], nbe[r]), k == 0);
        }
    const float Z = nal[1];
    const float freq_f = static_cast<float>(a.freq[i]);
    const uint32_t bucket = a.mode == SPM_ESTEP_PARITY ? BucketOf(a, i) : 0;
    uint64_t w = a.mode == SPM_ESTEP_PARITY ? a.rec_off[i] : 0;
    for (uint32_t p = 0; p < nc; ++p)
      for (int32_t k = 0; k < bcount[p]; ++k) {
        const int32_t nd = begin_list(p, k);
        const float ex = __fsub_rn(__fadd_rn(__fadd_rn(nal[nd], nscore[nd]), nbe[nd]), Z);
        if (a.mode == SPM_ESTEP_PARITY) {
          const uint32_t key = bucket * a.V + static_cast<uint32_t>(nid[nd]);
          if (a.exs) StoreRecordEx(a, w, key, ex);  // (kept: kept[i] = N[i] for this sentence)
          else StoreRecord(a, w, key, static_cast<double>(freq_f) * exp(static_cast<double>(ex)));
          ++w;
        } else {
          atomicAdd(&a.acc[nid[nd]], static_cast<double>(freq_f) * exp(static_cast<double>(ex)));
        }
      }
    // Viterbi size (unigram_model.cc:222-261)
    for (uint32_t p = 0; p <= nc; ++p)
      for (int32_t k = 0; k < bcount[p]; ++k) {
        const int32_t r = begin_list(p, k);
        float best_score = 0.f;
        int32_t best = -1;
        for (int32_t l = end_head[p]; l >= 0; l = nnext[l]) {
          const float sc = __fadd_rn(nbt[l], nscore[r]);
          if (best < 0 || sc > best_score) {
            best = l;
            best_score = sc;
          }
        }
        nprev[r] = best;
        nbt[r] = best_score;
      }
    uint32_t k = 0;
    for (int32_t nd = nprev[1]; nd >= 0 && nprev[nd] >= 0; nd = nprev[nd]) ++k;
    a.Zlat[i] = Z;
    a.ntok[i] = k;
    if (a.mode == SPM_ESTEP_FAST) {
      atomicAdd(a.acc_obj, -static_cast<double>(__fdiv_rn(__fmul_rn(freq_f, Z), a.all_freq_f)));
      atomicAdd(reinterpret_cast<unsigned long long *>(a.ntok_b), static_cast<unsigned long long>(k));
    }
  }
}

// Pieces of 32+ chars (no register ring): every sentence takes the general
// kernel.  This pre-pass lists them on the device and counts each one's
// lattice nodes exactly as estep_general_kernel inserts them (trie leaves
// per char start, byte-wise, plus the UNK node when no 1-char piece starts
// there; unigram_model.cc:535-604), so PARITY records get their offsets.
__global__ __launch_bounds__(256) void estep_count_kernel(EArgs a) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t b0 = a.off[i];
  const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
  const uint8_t *__restrict__ s = a.bytes + b0;
  uint32_t nodes = 0;
  for (uint32_t p = 0; p < nb;) {
    uint32_t cl = OneCharLenDev(s[p]);
    if (cl > nb - p) cl = nb - p;
    const uint32_t first_end = p + cl;
    bool single = false;
    uint32_t base = a.root_base;
    for (uint32_t q = p; q < nb; ++q) {
      const uint32_t c = s[q];
      if (c == 0) break;
      const uint32_t u = a.units[base ^ c];
      if ((u & 0xFFu) != c) break;
      base = u >> 9;
      if (u & 0x100u) {
        ++nodes;
        if (q + 1 <= first_end) single = true;  // ends inside the first char: length 1
      }
    }
    if (!single) ++nodes;
    p = first_end;
  }
  a.N[i] = nodes;
  a.ntok[i] = kNone;
  a.flagged[i] = static_cast<uint32_t>(i);
  atomicMax(&a.status[1], nb);
  if (i == 0) a.status[0] = static_cast<uint32_t>(a.n);
}

// status[3] |= 1 if some sentence freq of the chunk is negative (the record
// drop below needs non-negative contributions).
__global__ __launch_bounds__(256) void estep_freq_check_kernel(const int64_t *__restrict__ freq, uint64_t n,
                                                               uint32_t *__restrict__ status) {
  bool neg = false;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    neg |= freq[i] < 0;
  if (__ballot(neg) && (threadIdx.x & 63) == 0) atomicOr(&status[3], 1u);
}

// PARITY record drop.  Every accumulator is the float chain
// e = (float)((double)e + c) over records c = freq * exp(...) >= 0 from a
// zeroed start, so it never decreases and any value read earlier is a lower
// bound e_lb <= e.  For a positive normal e_lb with biased exponent x,
// ulp(e) >= ulp(e_lb) = 2^(x - 150); a record c < 2^(x - 152) (a quarter of
// that) gives a double sum within ulp/4 + 2^-29 ulp of e, which the float
// rounding returns to e exactly: the record is a no-op and is not written.
// Per hot piece (kHot highest scores, the pieces with most records), the
// bound's exponent is the minimum over the buckets this call touches
// (b = r0 (mod g)); 0 = no bound (zero, denormal, inf/NaN or negative).
// The accumulators may be mid-fold on the side stream: a 32-bit float read
// returns some value of the chain, still a lower bound.
__global__ __launch_bounds__(256) void estep_threshold_kernel(const float *__restrict__ expb, uint64_t V, int T,
                                                              uint32_t r0, uint32_t g,
                                                              const int32_t *__restrict__ hot_id, uint32_t nhot,
                                                              uint8_t *__restrict__ drop_exp) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= kHot) return;
  uint32_t m = 0;
  if (s < nhot) {
    const uint64_t id = static_cast<uint64_t>(hot_id[s]);
    m = 0xFFu;
    for (uint32_t t = r0; t < static_cast<uint32_t>(T); t += g) {
      const uint32_t b = __float_as_uint(expb[static_cast<uint64_t>(t) * V + id]);
      const uint32_t x = (b >> 23) & 0xFFu;
      m = min(m, (b >> 31) || x == 0xFFu ? 0u : x);
    }
    if (m == 0xFFu) m = 0;
  }
  drop_exp[s] = static_cast<uint8_t>(m);
}

// PARITY: the records a sentence kept are the last kept[i] slots of its range
// [rec_off[i], rec_off[i] + N[i]); copy them, in order, to their place in the
// dense list (koff = exclusive scan of kept).  One wavefront per 64
// consecutive sentences walks the wave's output range [koff[i0],
// koff[i0 + 64]) with consecutive lanes on consecutive records (coalesced
// stores; the loads are runs per sentence); each record's sentence comes
// from a binary search over the wave's 64 koff values held one per lane.
__global__ __launch_bounds__(256) void estep_compact_records_kernel(uint64_t n, const uint64_t *__restrict__ rec_off,
                                                                    const uint32_t *__restrict__ N,
                                                                    const uint32_t *__restrict__ kept,
                                                                    const uint64_t *__restrict__ koff,
                                                                    const uint32_t *__restrict__ keys_in,
                                                                    const double *__restrict__ vals_in,
                                                                    const float *__restrict__ exs_in,
                                                                    const int64_t *__restrict__ freq,
                                                                    uint32_t *__restrict__ keys_out,
                                                                    double *__restrict__ vals_out,
                                                                    const uint2 *__restrict__ RT,
                                                                    const uint16_t *__restrict__ colmap,
                                                                    uint32_t rt_rows) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t i0 = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) & ~63ull;
  if (i0 >= n) return;
  const uint64_t i = i0 + lane;
  const uint32_t cnt = static_cast<uint32_t>(n - i0 < 64 ? n - i0 : 64);
  // Lane l: its sentence's first output slot and its first kept source record.
  const uint64_t kfirst = i < n ? koff[i] : koff[n];
  const uint32_t kc_i = i < n ? kept[i] : 0;
  const uint64_t src0 = i < n ? rec_off[i] + N[i] - kc_i : 0;
  const uint64_t obeg = __shfl(kfirst, 0), oend = koff[i0 + cnt];
  // RT (tile-transposed records): lane l's sentence's column in its tile.
  // (General-path sentences: 0xFFFF, records in range slots.)
  const uint32_t col_i = RT && i < n ? colmap[i] : 0xFFFFu;
  // Every lane stays active through the loop (the shuffles read other
  // lanes' registers); only the copy itself is guarded.
  for (uint64_t jb = obeg; jb < oend; jb += 64) {
    const uint64_t j = jb + lane;
    // Last sentence s of the wave with koff[s] <= j (a sentence's kept
    // records are [koff[s], koff[s + 1]); empty ones share the next koff,
    // and the search takes the last of equal values).  Fixed 6 steps.
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 32; step >= 1; step >>= 1) {
      const uint32_t cand = lo + step;
      const uint64_t kc = __shfl(kfirst, static_cast<int>(cand < 64 ? cand : 63));
      if (cand < cnt && kc <= j) lo = cand;
    }
    const uint64_t r = j - __shfl(kfirst, static_cast<int>(lo));  // record r of the sentence's kept ones
    const uint64_t src = __shfl(src0, static_cast<int>(lo)) + r;
    const uint32_t kept_s = __shfl(kc_i, static_cast<int>(lo));
    const uint32_t col_s = __shfl(col_i, static_cast<int>(lo));
    if (j < oend) {
      const uint64_t k = static_cast<uint64_t>(kept_s) - 1 - r;  // its keep order (0 = last slot)
      if (col_s != 0xFFFFu && k < rt_rows) {
        const uint64_t s_abs = i0 + lo;
        const uint2 x = RT[((s_abs >> 8) * rt_rows + k) * 256 + col_s];
        keys_out[j] = x.x;
        vals_out[j] = static_cast<double>(static_cast<float>(freq[s_abs])) * exp(static_cast<double>(__uint_as_float(x.y)));
      } else {
        keys_out[j] = keys_in[src];
        // Deferred values: c = (double)freq * exp((double)ex), the walk's
        // formula, for the kept records only.
        vals_out[j] = exs_in ? static_cast<double>(static_cast<float>(freq[i0 + lo])) *
                                   exp(static_cast<double>(exs_in[src]))
                             : vals_in[src];
      }
    }
  }
}

// PARITY: seg[k] = first record with key >= k in the sorted keys (k <= nkeys).
__global__ __launch_bounds__(256) void estep_seg_bounds_kernel(const uint32_t *__restrict__ keys,
                                                               uint64_t nrec, uint64_t nkeys,
                                                               uint64_t *__restrict__ seg) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k > nkeys) return;
  uint64_t lo = 0, hi = nrec;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  seg[k] = lo;
}

// PARITY folds.  Per (bucket, id) key, e = (float)((double)e + c) over its
// records in order (the sort is stable, records were written in reference
// order: expected[n][id] += freq * exp(...), unigram_model.cc:318-326 with
// the per-thread vectors of unigram_model_trainer.cc:237-287); per bucket,
// objs[t] -= Z / all_sentence_freq in sentence order (:266-270).
//
// The float recurrence is sequential, but it is linear inside a binade.  While
// e is a normal float in [2^k, 2^(k+1)), e = m*u (u = 2^(k-23), m < 2^24) and
// the double sum is fl64(e + c) = e + rne_g(c) with g = u*2^-29 (e/g is even,
// so ties-to-even of the sum equal those of c/g alone).  The float rounding
// then adds d(c) = round(rne_g(c)/u) ulps -- independent of e -- unless that
// quotient ends in exactly .5: then ties-to-even rounds to the even mantissa,
// d = floor + ((m' + floor) & 1) with m' the running mantissa, and the
// mantissa is even afterwards.  So only the parity of m' matters: a record
// maps parity p to p ^ (d & 1), a tie maps it to 0; those maps compose, and
// a wave scan of them gives every tie its d (exact contributions such as
// freq * exp(0) = 1.0 are ties once e reaches 2^24).  A record whose sum
// leaves the binade (m + d reaches 2^24) is an "event".  A wavefront takes
// 64*kFoldR records per window, computes every d, scans them, applies all
// records before the first event in closed form (e = (m + prefix)*u, exact)
// and runs the event record with the sequential rule.  e outside the normal
// positive range (0 at the start, denormals, inf/NaN) and negative or NaN
// contributions also take the sequential rule.  A key with n records thus
// costs ~n/(64*kFoldR) windows plus one step per binade crossing instead of n
// dependent fp64 adds.
constexpr uint32_t kFoldCap = 1u << 26;  // saturating ulp counts (>= 2^24 is a crossing)

__device__ __forceinline__ uint32_t SatAdd(uint32_t a, uint32_t b) { return min(a + b, kFoldCap); }

// Element j of the chain is vals[j * stride], j in [p, end); kFoldR records
// per lane and window.
template <int kFoldR>
__device__ float FoldKey(const double *__restrict__ vals, uint64_t p, const uint64_t end, float e,
                         const uint32_t lane, const uint64_t stride = 1) {
  double cur[kFoldR], nxt[kFoldR];
  uint64_t cur_at = ~0ull;  // window start the `cur` values belong to
  while (p < end) {
    const uint32_t eb = __float_as_uint(e);
    const uint32_t ex = (eb >> 23) & 0xFFu;
    if (ex == 0 || ex == 0xFFu || (eb >> 31)) {
      e = static_cast<float>(__dadd_rn(static_cast<double>(e), vals[p * stride]));
      ++p;
      continue;
    }
    if (cur_at != p) {
#pragma unroll
      for (int s = 0; s < kFoldR; ++s) {
        const uint64_t q = p + lane * kFoldR + s;
        cur[s] = q < end ? vals[q * stride] : 0.0;
      }
    }
    // Prefetch the window that follows if this one has no event.
    const uint64_t pn = p + 64 * kFoldR;
#pragma unroll
    for (int s = 0; s < kFoldR; ++s) {
      const uint64_t q = pn + lane * kFoldR + s;
      nxt[s] = q < end ? vals[q * stride] : 0.0;
    }
    const int k = static_cast<int>(ex) - 127;
    const uint32_t m = (eb & 0x7FFFFFu) | 0x800000u;
    const double to_g = __builtin_ldexp(1.0, 52 - k);  // c / g
    uint32_t dv[kFoldR];
    uint32_t tie_mask = 0, bad_mask = 0;
    // Lane parity function of its records: a tie leaves an even mantissa
    // (reset to 0), any other record flips the parity by d & 1.
    uint32_t fr_reset = 0, fr_x = 0;
#pragma unroll
    for (int s = 0; s < kFoldR; ++s) {
      const uint64_t q = p + lane * kFoldR + s;
      uint32_t d = 0;
      if (q < end) {
        const double c = cur[s];
        const double x = c * to_g;
        if (!(c >= 0.0) || !(x < 9007199254740992.0)) {  // negative/NaN, or c >= 2^(k+1)
          d = kFoldCap;
          bad_mask |= 1u << s;
        } else {
          const double y = __builtin_rint(x) * 0x1p-29;
          const double fl = __builtin_floor(y);
          const double fr = y - fl;
          d = static_cast<uint32_t>(fl);
          if (fr == 0.5) {
            tie_mask |= 1u << s;
            fr_reset = 1;
            fr_x = 0;
          } else {
            d += fr > 0.5 ? 1u : 0u;
            fr_x ^= d & 1u;
          }
        }
      }
      dv[s] = d;
    }
    // Exclusive wave scan of the parity functions (f2 after f1: f2 if it
    // resets, else (f1.reset, f1.x ^ f2.x)), then each tie's rounding
    // direction: ties-to-even on the running mantissa m + prefix.
    uint32_t sr = fr_reset, sx = fr_x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t r2 = __shfl_up(sr, off), x2 = __shfl_up(sx, off);
      if (lane >= static_cast<uint32_t>(off) && !sr) {
        sr = r2;
        sx ^= x2;
      }
    }
    uint32_t er = __shfl_up(sr, 1), ex2 = __shfl_up(sx, 1);
    if (lane == 0) er = ex2 = 0;
    uint32_t par = er ? ex2 : ((m & 1u) ^ ex2);
    uint32_t pre[kFoldR];
    uint32_t acc = 0;
#pragma unroll
    for (int s = 0; s < kFoldR; ++s) {
      const uint64_t q = p + lane * kFoldR + s;
      if (q < end && !((bad_mask >> s) & 1u)) {
        if ((tie_mask >> s) & 1u) {
          dv[s] += (par + dv[s]) & 1u;
          par = 0;
        } else {
          par ^= dv[s] & 1u;
        }
      }
      acc = SatAdd(acc, dv[s]);
      pre[s] = acc;
    }
    // Wave inclusive scan of the lane totals (saturating add is associative).
    uint32_t incl = acc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(incl, off);
      if (lane >= static_cast<uint32_t>(off)) incl = SatAdd(incl, t);
    }
    uint32_t excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0;
    // First event of this lane and the exact ulp count before it.
    int ev = kFoldR;
    uint32_t before = 0;
#pragma unroll
    for (int s = kFoldR - 1; s >= 0; --s) {
      const uint64_t q = p + lane * kFoldR + s;
      const uint32_t inc = SatAdd(excl, pre[s]);
      const bool crossing = m + inc >= (1u << 24);
      if (q < end && (((bad_mask >> s) & 1u) || crossing)) {
        ev = s;
        before = s == 0 ? excl : SatAdd(excl, pre[s > 0 ? s - 1 : 0]);
      }
    }
    const uint64_t bal = __ballot(ev < kFoldR);
    if (bal == 0) {
      const uint32_t total = __shfl(incl, 63);  // m + total < 2^24: no crossing in the window
      e = __builtin_ldexpf(static_cast<float>(m + total), k - 23);
      p = min(pn, end);
#pragma unroll
      for (int s = 0; s < kFoldR; ++s) cur[s] = nxt[s];
      cur_at = p;
    } else {
      const int L = __ffsll(static_cast<unsigned long long>(bal)) - 1;
      const int s = __shfl(ev, L);
      const uint32_t b = __shfl(before, L);  // m + b < 2^24 (no earlier event)
      const float e0 = __builtin_ldexpf(static_cast<float>(m + b), k - 23);
      const uint64_t q = p + static_cast<uint64_t>(L) * kFoldR + s;
      e = static_cast<float>(__dadd_rn(static_cast<double>(e0), vals[q * stride]));
      p = q + 1;
    }
  }
  return e;
}

// PARITY obj records: q[i] = -(float)((freq * Z) / all_sentence_freq) as a
// double (objs[t] -= Z / all_sentence_freq, unigram_model_trainer.cc:266-270,
// is a float chain o = fl32(o + q); for float q the double-then-float
// rounding of FoldKey equals that single rounding), and ntok per bucket
// (integer, order-free) through per-block LDS sums.
__global__ __launch_bounds__(256) void estep_objq_kernel(EArgs a, double *__restrict__ objq) {
  __shared__ unsigned long long nt[128];
  for (int t = threadIdx.x; t < a.T; t += blockDim.x) nt[t] = 0;
  __syncthreads();
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.n) {
    const float q = __fdiv_rn(__fmul_rn(static_cast<float>(a.freq[i]), a.Zlat[i]), a.all_freq_f);
    objq[i] = -static_cast<double>(q);
    atomicAdd(&nt[BucketOf(a, i)], static_cast<unsigned long long>(a.ntok[i]));
  }
  __syncthreads();
  for (int t = threadIdx.x; t < a.T; t += blockDim.x)
    if (nt[t]) atomicAdd(reinterpret_cast<unsigned long long *>(a.ntok_b + t), nt[t]);
}

// Bucket t's sentences of this call form one arithmetic progression:
// (index_base + k * index_stride) mod T == t for k = k0, k0 + step, ... with
// step = T / gcd(index_stride mod T, T).
template <int kFoldR>
__device__ void FoldObj(const EArgs &a, const uint32_t t, const uint32_t lane, const double *__restrict__ objq,
                        float *__restrict__ objb) {
  const uint64_t T = static_cast<uint64_t>(a.T);
  uint64_t k0 = T;
  for (uint64_t k = 0; k < T; ++k)
    if (BucketOf(a, k) == t) {
      k0 = k;
      break;
    }
  if (k0 >= T || k0 >= a.n) return;
  uint64_t g = T, r = a.index_stride % T;
  while (r) {
    const uint64_t x = g % r;
    g = r;
    r = x;
  }
  const uint64_t step = T / g;
  const uint64_t cnt = (a.n - k0 + step - 1) / step;
  const float o = FoldKey<kFoldR>(objq + k0, 0, cnt, objb[t], lane, step);
  if (lane == 0) objb[t] = o;
}

// Keys by record count: "heavy" (more than kLightMax records) get a
// wavefront each (FoldKey's windows), "light" ones a lane each (a short
// sequential fold), empty ones nothing.
constexpr uint32_t kLightMax = 64;

__global__ __launch_bounds__(256) void estep_classify_kernel(const uint64_t *__restrict__ seg, uint64_t nkeys,
                                                             uint32_t *__restrict__ heavy,
                                                             uint32_t *__restrict__ light,
                                                             uint32_t *__restrict__ counts) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t c = k < nkeys ? seg[k + 1] - seg[k] : 0;
  const bool h = c > kLightMax, l = c > 0 && !h;
  // One atomic per wave and list (512 k keys on two counters would serialise).
  const uint64_t bh = __ballot(h), bl = __ballot(l);
  const uint64_t below = (1ull << lane) - 1;
  uint32_t oh = 0, ol = 0;
  if (lane == 0) {
    if (bh) oh = atomicAdd(&counts[0], static_cast<uint32_t>(__popcll(bh)));
    if (bl) ol = atomicAdd(&counts[1], static_cast<uint32_t>(__popcll(bl)));
  }
  oh = __shfl(oh, 0);
  ol = __shfl(ol, 0);
  if (h) heavy[oh + __popcll(bh & below)] = static_cast<uint32_t>(k);
  if (l) light[ol + __popcll(bl & below)] = static_cast<uint32_t>(k);
}

// Blocks [0, T): the obj chains; the other G = gridDim.x - T blocks take the
// heavy keys (one wavefront per key) and then the light keys (one lane per
// key) grid-stride.  The list sizes are read on the device (counts[0] heavy,
// counts[1] light), so the launch needs no host read-back and the fold stays
// queued behind the sort on the side stream.
template <int kFoldR>
__global__ __launch_bounds__(64) void estep_fold_kernel(EArgs a, const double *__restrict__ objq,
                                                        float *__restrict__ objb,
                                                        const uint64_t *__restrict__ seg,
                                                        const double *__restrict__ vals,
                                                        float *__restrict__ expb,
                                                        const uint32_t *__restrict__ heavy,
                                                        const uint32_t *__restrict__ light,
                                                        const uint32_t *__restrict__ counts) {
  const uint32_t lane = threadIdx.x;
  const uint32_t T = static_cast<uint32_t>(a.T);
  if (blockIdx.x < T) {
    FoldObj<kFoldR>(a, blockIdx.x, lane, objq, objb);
    return;
  }
  const uint32_t G = gridDim.x - T, g = blockIdx.x - T;
  const uint32_t nh = counts[0], nl = counts[1];
  for (uint32_t h = g; h < nh; h += G) {
    const uint32_t key = heavy[h];
    const float e = FoldKey<kFoldR>(vals, seg[key], seg[key + 1], expb[key], lane);
    if (lane == 0) expb[key] = e;
  }
  for (uint64_t j = static_cast<uint64_t>(g) * 64 + lane; j < nl; j += static_cast<uint64_t>(G) * 64) {
    const uint32_t key = light[j];
    uint64_t p = seg[key];
    const uint64_t end = seg[key + 1];
    float e = expb[key];
    for (; p + 8 <= end; p += 8) {
      double v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = vals[p + t];
#pragma unroll
      for (int t = 0; t < 8; ++t) e = static_cast<float>(__dadd_rn(static_cast<double>(e), v[t]));
    }
    for (; p < end; ++p) e = static_cast<float>(__dadd_rn(static_cast<double>(e), vals[p]));
    expb[key] = e;
  }
}

__global__ void estep_finalize_kernel(int mode, int T, uint64_t V, const double *__restrict__ acc,
                                      const double *__restrict__ acc_obj,
                                      const float *__restrict__ expb, const float *__restrict__ objb,
                                      const int64_t *__restrict__ ntok_b, float *__restrict__ expected,
                                      float *__restrict__ obj, int64_t *__restrict__ ntok) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k < V) {
    if (mode == SPM_ESTEP_FAST) {
      expected[k] = static_cast<float>(acc[k]);
    } else {
      float e = expb[k];
      for (int t = 1; t < T; ++t) e = __fadd_rn(e, expb[static_cast<uint64_t>(t) * V + k]);
      expected[k] = e;
    }
  }
  if (k == 0) {
    if (mode == SPM_ESTEP_FAST) {
      *obj = static_cast<float>(*acc_obj);
      *ntok = ntok_b[0];
    } else {
      float o = objb[0];
      int64_t nt = ntok_b[0];
      for (int t = 1; t < T; ++t) {
        o = __fadd_rn(o, objb[t]);
        nt += ntok_b[t];
      }
      *obj = o;
      *ntok = nt;
    }
  }
}

// ---------------------------------------------------------------------------
// NBest(2) of the pruning step (unigram_model_trainer.cc:348-371 over
// Lattice::NBest, unigram_model.cc:339-477), one piece per lane: the lattice
// of the piece's own string under the TrainerModel (unk id 0 at min_score -
// 10, every piece NORMAL), Viterbi (strict >, first lnode wins), then the A*
// agenda as a binary heap with libstdc++'s push_heap / pop_heap moves
// (std::priority_queue<Hypothesis*> ordered by fx <) so equal-fx hypotheses
// pop in the reference's order.  A piece whose hypotheses outgrow the slab is
// flagged (keep = 2) for the host path.
// ---------------------------------------------------------------------------
struct NBestArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  uint64_t V;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;
  const float *__restrict__ scores;
  uint32_t root_base;
  float unk_score;
  uint8_t *__restrict__ scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;
  int K;
  uint32_t max_hyps;
  uint8_t *__restrict__ keep;    // 0 / 1, 2 = redo on the host
  int32_t *__restrict__ alt;     // alternatives (ids of the second best path)
  const uint64_t *__restrict__ alt_off;
  uint32_t *__restrict__ alt_n;
};

uint64_t NBestSlab(uint32_t nb, int K, uint32_t max_hyps) {
  const uint64_t cap = static_cast<uint64_t>(nb) * K + 2;
  return ((static_cast<uint64_t>(nb) + 1) * 5 + cap * 7 + static_cast<uint64_t>(max_hyps) * 5) * 4 + 64;
}

__global__ __launch_bounds__(64) void prune_nbest_kernel(NBestArgs g) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = tid; i < g.V; i += nthreads) {
    const uint64_t b0 = g.off[i];
    const uint32_t nb = static_cast<uint32_t>(g.off[i + 1] - b0);
    g.alt_n[i] = 0;
    if (nb > g.max_nb || nb == 0) {
      g.keep[i] = 2;
      continue;
    }
    const uint8_t *__restrict__ s = g.bytes + b0;
    uint8_t *slab = g.scratch + tid * g.slab_bytes;
    const uint32_t cap = nb * g.K + 2;
    uint32_t *cs = reinterpret_cast<uint32_t *>(slab);
    int32_t *end_head = reinterpret_cast<int32_t *>(cs + nb + 1);
    int32_t *end_tail = end_head + nb + 1;
    int32_t *bfirst = end_tail + nb + 1;
    int32_t *bcount = bfirst + nb + 1;
    float *nscore = reinterpret_cast<float *>(bcount + nb + 1);
    float *nbt = nscore + cap;
    int32_t *nid = reinterpret_cast<int32_t *>(nbt + cap);
    int32_t *nprev = nid + cap;
    int32_t *nnext = nprev + cap;
    uint32_t *npos = reinterpret_cast<uint32_t *>(nnext + cap);
    uint32_t *nlen = npos + cap;
    int32_t *hnode = reinterpret_cast<int32_t *>(nlen + cap);
    int32_t *hnext = hnode + g.max_hyps;
    float *hfx = reinterpret_cast<float *>(hnext + g.max_hyps);
    float *hgx = hfx + g.max_hyps;
    int32_t *heap = reinterpret_cast<int32_t *>(hgx + g.max_hyps);
    // SetSentence + PopulateNodes (unigram_model.cc:147-187, 535-604).
    uint32_t nc = 0;
    for (uint32_t q = 0; q < nb;) {
      cs[nc++] = q;
      const uint32_t cl = OneCharLenDev(s[q]);
      q += cl < nb - q ? cl : nb - q;
    }
    cs[nc] = nb;
    for (uint32_t p = 0; p <= nc; ++p) {
      end_head[p] = end_tail[p] = -1;
      bfirst[p] = bcount[p] = 0;
    }
    auto push_end = [&](uint32_t q, int32_t nd) {
      nnext[nd] = -1;
      if (end_tail[q] < 0) end_head[q] = nd;
      else nnext[end_tail[q]] = nd;
      end_tail[q] = nd;
    };
    auto init_node = [&](int32_t nd, uint32_t p, uint32_t len, int32_t id, float sc) {
      nscore[nd] = sc;
      nbt[nd] = 0.f;
      nid[nd] = id;
      nprev[nd] = -1;
      npos[nd] = p;
      nlen[nd] = len;
    };
    init_node(0, 0, 0, -1, 0.f);  // BOS
    push_end(0, 0);
    init_node(1, nc, 0, -1, 0.f);  // EOS
    int32_t nn = 2;
    bfirst[nc] = 1;
    bcount[nc] = 1;
    for (uint32_t p = 0; p < nc; ++p) {
      bfirst[p] = nn;
      bool single = false;
      uint32_t base = g.root_base, cpos = p;
      for (uint32_t q = cs[p]; q < nb; ++q) {
        const uint32_t c = s[q];
        if (c == 0) break;
        const uint32_t node = base ^ c;
        const uint32_t u = g.units[node];
        if ((u & 0xFFu) != c) break;
        base = u >> 9;
        if (u & 0x100u) {
          while (cs[cpos] < q + 1) ++cpos;
          const uint32_t length = cpos - p;
          const int32_t id = g.values[node];
          const int32_t nd = nn++;
          init_node(nd, p, length, id, g.scores[id]);
          push_end(p + length, nd);
          if (length == 1) single = true;
        }
      }
      if (!single) {
        const int32_t nd = nn++;
        init_node(nd, p, 1, 0, g.unk_score);
        push_end(p + 1, nd);
      }
      bcount[p] = nn - bfirst[p];
    }
    // Viterbi (unigram_model.cc:222-261).
    for (uint32_t p = 0; p <= nc; ++p)
      for (int32_t k = 0; k < bcount[p]; ++k) {
        const int32_t r = bfirst[p] + k;
        int32_t best = -1;
        float best_score = 0.f;
        for (int32_t l = end_head[p]; l >= 0; l = nnext[l]) {
          const float sc = __fadd_rn(nbt[l], nscore[r]);
          if (best < 0 || sc > best_score) {
            best = l;
            best_score = sc;
          }
        }
        nprev[r] = best;
        nbt[r] = best_score;
      }
    // A* (unigram_model.cc:398-470).  libstdc++ heap moves, comp = fx <.
    uint32_t hn = 0, hs = 0;
    auto less = [&](int32_t x, int32_t y) { return hfx[x] < hfx[y]; };
    auto sift_up = [&](uint32_t hole, uint32_t top, int32_t v) {  // __push_heap
      uint32_t parent = hole > 0 ? (hole - 1) / 2 : 0;
      while (hole > top && less(heap[parent], v)) {
        heap[hole] = heap[parent];
        hole = parent;
        parent = hole > 0 ? (hole - 1) / 2 : 0;
      }
      heap[hole] = v;
    };
    auto push = [&](int32_t h) {
      heap[hs] = h;
      sift_up(hs, 0, h);
      ++hs;
    };
    auto pop = [&]() {  // pop_heap + pop_back
      if (hs > 1) {
        const uint32_t len = hs - 1;
        const int32_t v = heap[len];
        heap[len] = heap[0];
        uint32_t hole = 0, child = 0;
        while (child < (len - 1) / 2) {  // __adjust_heap
          child = 2 * (child + 1);
          if (less(heap[child], heap[child - 1])) --child;
          heap[hole] = heap[child];
          hole = child;
        }
        if ((len & 1u) == 0 && child == (len - 2) / 2) {
          child = 2 * (child + 1);
          heap[hole] = heap[child - 1];
          hole = child - 1;
        }
        sift_up(hole, 0, v);
      }
      --hs;
    };
    bool overflow = false;
    hnode[0] = 1;  // EOS
    hnext[0] = -1;
    hfx[0] = nscore[1];
    hgx[0] = nscore[1];
    hn = 1;
    push(0);
    int results = 0;
    uint32_t first_size = 0;
    while (hs > 0) {
      const int32_t top = heap[0];
      pop();
      if (hnode[top] == 0) {  // BOS: a complete path
        uint32_t sz = 0;
        for (int32_t h = hnext[top]; hnext[h] != -1; h = hnext[h]) {
          if (results == 1) g.alt[g.alt_off[i] + sz] = nid[hnode[h]];
          ++sz;
        }
        if (results == 0) first_size = sz;
        else g.alt_n[i] = sz;
        if (++results == 2) break;
        continue;
      }
      const int32_t tn = hnode[top];
      for (int32_t l = end_head[npos[tn]]; l >= 0; l = nnext[l]) {
        if (hn >= g.max_hyps) {
          overflow = true;
          break;
        }
        hnode[hn] = l;
        hnext[hn] = top;
        hfx[hn] = __fadd_rn(nbt[l], hgx[top]);
        hgx[hn] = __fadd_rn(nscore[l], hgx[top]);
        push(static_cast<int32_t>(hn));
        ++hn;
      }
      if (overflow) break;
    }
    // PruneSentencePieces (unigram_model_trainer.cc:355-370).
    if (overflow) {
      g.keep[i] = 2;
      g.alt_n[i] = 0;
    } else if (results == 1) {
      g.keep[i] = 1;
      g.alt_n[i] = 0;
    } else if (first_size >= 2) {
      g.keep[i] = 0;
      g.alt_n[i] = 0;
    } else {
      g.keep[i] = 1;
      if (first_size != 1) g.alt_n[i] = 0;
    }
  }
}

uint64_t EGeneralSlab(uint32_t nb, int K) {
  const uint64_t cap = static_cast<uint64_t>(nb) * K + 2;
  return ((static_cast<uint64_t>(nb) + 1) * 5 + cap * 9) * 4 + 64;
}

int Err(spm_hip_pieces *p, int code, const std::string &m) {
  p->last_error = m;
  return code;
}

#define E_TRY(expr)                                                               \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess)                                                         \
      return Err(P, SPM_INTERNAL, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

}  // namespace
}  // namespace spm_amd

using spm_amd::DevBuf;

namespace spm_amd {
namespace {
// One timing event on the caller's stream (spm_hip_pieces_set_timing).
void ETimingMark(spm_hip_pieces *P, hipStream_t st) {
  if (!P->timing) return;
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return;
  if (hipEventRecord(e, st) != hipSuccess) {
    (void)hipEventDestroy(e);
    return;
  }
  P->tev.push_back(e);
}
}  // namespace
}  // namespace spm_amd

extern "C" {

namespace {

// The score-dependent part of a piece set: TrainerModel's min score, unk
// score and tie bound, the kHot highest-score pieces, the per-unit leaf score
// and the walks' interleaved tables, uploaded.  The trie is P's.
bool PiecesScoreTables(spm_hip_pieces *P, const float *scores) {
  const uint64_t V = P->V;
  P->min_score = FLT_MAX;
  float mag = 0.f;
  for (uint64_t k = 0; k < V; ++k) {
    P->min_score = std::min(P->min_score, scores[k]);
    mag = std::max(mag, std::fabs(scores[k]));
  }
  // TrainerModel: min_score_ over the list, unk penalty 10 (unigram_model.cc:563).
  P->unk_score = P->min_score - 10.0f;
  P->tie_mag = std::max(mag, std::fabs(P->unk_score)) + 2.0f;
  if (!P->enc_off.empty()) P->enc_scores.assign(scores, scores + V);
  auto up = [&](spm_amd::DevBuf *b, const void *src, size_t bytes) -> bool {
    return b->Reserve(std::max<size_t>(bytes, 4)) == hipSuccess &&
           hipMemcpy(b->ptr, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  // Per-unit leaf score (unit → score in one load instead of values → scores),
  // and the walks' interleaved tables (EArgs::uvs / uvis).
  const size_t NU = P->trie.units.size();
  std::vector<float> vscore(NU, 0.f);
  for (size_t u = 0; u < NU; ++u)
    if (spm_amd::DoubleArray::Leaf(P->trie.units[u]) && P->trie.values[u] >= 0)
      vscore[u] = scores[P->trie.values[u]];
  // The kHot highest-score pieces: FAST-mode LDS privatisation and the
  // PARITY record drop's bound table.  (Score descending, index ascending: a
  // strict order, so selecting the first H and sorting only those equals a
  // stable sort's first H.)
  std::vector<int32_t> order(V);
  for (uint64_t k = 0; k < V; ++k) order[k] = static_cast<int32_t>(k);
  const uint64_t H = std::min<uint64_t>(V, spm_amd::kHotPieces);
  auto hotter = [&](int32_t x, int32_t y) { return scores[x] > scores[y] || (scores[x] == scores[y] && x < y); };
  if (H < V) std::nth_element(order.begin(), order.begin() + static_cast<std::ptrdiff_t>(H), order.end(), hotter);
  std::sort(order.begin(), order.begin() + static_cast<std::ptrdiff_t>(H), hotter);
  std::vector<int16_t> hot_slot(V, -1);
  std::vector<int32_t> hot_id(spm_amd::kHotPieces, 0);
  for (uint64_t s = 0; s < H; ++s) {
    hot_slot[order[s]] = static_cast<int16_t>(s);
    hot_id[s] = order[s];
  }
  std::vector<uint32_t> uvs(2 * NU), uvis(4 * NU, 0u);
  for (size_t u = 0; u < NU; ++u) {
    uint32_t sb;
    std::memcpy(&sb, &vscore[u], 4);
    uvs[2 * u] = uvis[4 * u] = P->trie.units[u];
    uvs[2 * u + 1] = uvis[4 * u + 2] = sb;
    uvis[4 * u + 1] = static_cast<uint32_t>(P->trie.values[u]);
    // 4th word: the leaf piece's hot slot + 1 (PARITY record drop), else 0.
    if (spm_amd::DoubleArray::Leaf(P->trie.units[u]) && P->trie.values[u] >= 0 &&
        hot_slot[P->trie.values[u]] >= 0)
      uvis[4 * u + 3] = static_cast<uint32_t>(hot_slot[P->trie.values[u]]) + 1u;
  }
  return up(&P->d_hot_slot, hot_slot.data(), V * 2) && up(&P->d_hot_id, hot_id.data(), hot_id.size() * 4) &&
         up(&P->d_scores, scores, V * 4) && up(&P->d_vscore, vscore.data(), vscore.size() * 4) &&
         up(&P->d_uvs, uvs.data(), uvs.size() * 4) && up(&P->d_uvis, uvis.data(), uvis.size() * 4);
}

}  // namespace

int spm_hip_pieces_create(const uint8_t *piece_bytes, const uint64_t *piece_off, const float *scores,
                          uint64_t V, spm_hip_pieces **out) {
  if (!out || !piece_off || (V && (!piece_bytes || !scores))) return SPM_INVALID_ARGUMENT;
  *out = nullptr;
  if (V == 0 || V >= (1ull << 28)) return SPM_OUT_OF_RANGE;
  auto *P = new spm_hip_pieces();
  P->V = V;
  std::vector<std::pair<std::string, int32_t>> keys(V);
  int max_chars = 0;
  for (uint64_t k = 0; k < V; ++k) {
    keys[k].first.assign(reinterpret_cast<const char *>(piece_bytes) + piece_off[k],
                         piece_off[k + 1] - piece_off[k]);
    keys[k].second = static_cast<int32_t>(k);
    int c = 0;
    const std::string &s = keys[k].first;
    for (size_t q = 0; q < s.size() && s[q] != '\0';) {
      q += std::min<size_t>(spm_amd::OneCharLen(static_cast<uint8_t>(s[q])), s.size() - q);
      ++c;
    }
    max_chars = std::max(max_chars, c);
  }
  std::string err;
  if (!spm_amd::BuildDoubleArray(std::move(keys), &P->trie, &err)) {
    delete P;
    return SPM_RESOURCE_EXHAUSTED;
  }
  P->root_base = spm_amd::DoubleArray::Base(P->trie.units[0]);
  P->trie_results_size = P->trie.max_prefix_matches;
  P->ring_width = max_chars < 16 ? 16 : max_chars < 32 ? 32 : 0;
  // The byte kernel's E-step mode needs a TrainerModel that encodes with the
  // byte kernel (whole-char pieces of < 16 bytes).  It is built on the first
  // large accumulate call (its trie build would dominate the small E-steps of
  // spm_train over unique words), from this copy of the list.
  if (P->ring_width == 16) {
    P->enc_bytes.assign(reinterpret_cast<const char *>(piece_bytes), piece_off[V]);
    P->enc_off.assign(piece_off, piece_off + V + 1);
  }
  auto up = [&](spm_amd::DevBuf *b, const void *src, size_t bytes) -> bool {
    return b->Reserve(std::max<size_t>(bytes, 4)) == hipSuccess &&
           hipMemcpy(b->ptr, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!PiecesScoreTables(P, scores) ||
      !up(&P->d_units, P->trie.units.data(), P->trie.units.size() * 4) ||
      !up(&P->d_values, P->trie.values.data(), P->trie.values.size() * 4) ||
      hipHostMalloc(reinterpret_cast<void **>(&P->pinned), 64) != hipSuccess) {
    spm_hip_pieces_free(P);
    return SPM_INTERNAL;
  }
  *out = P;
  return SPM_OK;
}

int spm_hip_pieces_set_scores(spm_hip_pieces *P, const float *scores, uint64_t V) {
  if (!P || !scores) return SPM_INVALID_ARGUMENT;
  if (V != P->V) return SPM_OUT_OF_RANGE;
  std::lock_guard<std::recursive_mutex> lock(P->mu);  // host state shared with accumulate / finalize
  // Nothing of P's may be in flight: its fold stream drains here, the
  // caller's streams are the caller's to drain (spm_hip.h).
  if (P->fold_st && hipStreamSynchronize(P->fold_st) != hipSuccess) return SPM_INTERNAL;
  // The byte-kernel TrainerModel holds the old scores: rebuilt on next use.
  if (P->enc) spm_hip_model_free(P->enc);
  P->enc = nullptr;
  P->enc_tried = false;
  return PiecesScoreTables(P, scores) ? SPM_OK : SPM_INTERNAL;
}

void spm_hip_pieces_free(spm_hip_pieces *P) {
  if (!P) return;
  for (hipEvent_t e : P->tev) (void)hipEventDestroy(e);
  P->tev.clear();
  if (P->fold_st) (void)hipStreamSynchronize(P->fold_st);  // before its buffers go
  for (DevBuf *b : {&P->d_units, &P->d_values, &P->d_scores, &P->d_vscore, &P->d_uvs, &P->d_uvis, &P->d_hot_slot, &P->d_hot_id, &P->w_A, &P->w_Z, &P->w_N, &P->w_ntok,
                    &P->w_flag, &P->w_status, &P->w_recoff, &P->w_keys, &P->w_vals, &P->w_keys2,
                    &P->w_cls[0], &P->w_cls[1], &P->w_cnt, &P->w_seg, &P->w_tmp, &P->w_scratch, &P->w_bp,
                    &P->w_red, &P->w_objq, &P->w_svals[0], &P->w_svals[1], &P->w_sseg[0], &P->w_sseg[1],
                    &P->w_sobjq[0], &P->w_sobjq[1], &P->w_heavy[0], &P->w_heavy[1], &P->w_light[0],
                    &P->w_light[1], &P->w_drop, &P->w_kept, &P->w_koff, &P->w_ckeys, &P->w_cvals, &P->w_AT,
                    &P->w_lanemap, &P->w_colmap, &P->w_RT})
    b->Release();
  if (P->fold_st) {
    (void)hipStreamSynchronize(P->fold_st);
    (void)hipStreamDestroy(P->fold_st);
  }
  for (int k = 0; k < 2; ++k) {
    if (P->ev_ready[k]) (void)hipEventDestroy(P->ev_ready[k]);
    if (P->ev_done[k]) (void)hipEventDestroy(P->ev_done[k]);
  }
  if (P->pinned) (void)hipHostFree(P->pinned);
  P->w_ectl.Release();
  if (P->enc) spm_hip_model_free(P->enc);
  delete P;
}

int spm_hip_pieces_set_forward(spm_hip_pieces *P, int mode) {
  if (!P || mode < 0 || mode > 2) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  P->forward_mode = mode;
  return SPM_OK;
}

int spm_hip_estep_record_stats(spm_hip_pieces *P, uint64_t *written, uint64_t *kept) {
  if (!P || !written || !kept) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  *written = P->rec_total;
  *kept = P->rec_kept;
  return SPM_OK;
}

int spm_hip_pieces_set_timing(spm_hip_pieces *P, int enable) {
  if (!P) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  P->timing = enable != 0;
  return SPM_OK;
}

int spm_hip_estep_kernel_times(spm_hip_pieces *P, double *fwd_ms, double *bwd_ms, uint64_t *chunks) {
  if (!P || !fwd_ms || !bwd_ms || !chunks) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  double f = 0, b = 0;
  uint64_t c = 0;
  int rc = SPM_OK;
  for (size_t k = 0; k + 3 < P->tev.size(); k += 4) {
    float x = 0, y = 0;
    if (hipEventSynchronize(P->tev[k + 3]) != hipSuccess ||
        hipEventElapsedTime(&x, P->tev[k], P->tev[k + 1]) != hipSuccess ||
        hipEventElapsedTime(&y, P->tev[k + 2], P->tev[k + 3]) != hipSuccess)
      rc = SPM_INTERNAL;
    f += x;
    b += y;
    ++c;
  }
  for (hipEvent_t e : P->tev) (void)hipEventDestroy(e);
  P->tev.clear();
  *fwd_ms = f;
  *bwd_ms = b;
  *chunks = c;
  return rc;
}

const char *spm_hip_pieces_last_error(const spm_hip_pieces *P) {
  return P ? P->last_error.c_str() : "";
}

int spm_hip_estep_accumulate(spm_hip_pieces *P, const uint8_t *d_bytes, const uint64_t *d_off,
                             const int64_t *d_freq, uint64_t n, int64_t all_sentence_freq,
                             int mode, int T, uint64_t index_base, uint64_t index_stride,
                             void *d_acc, void *d_acc_obj, int64_t *d_ntok_acc, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_estep_accumulate");
  using namespace spm_amd;
  if (!P) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  const bool defer = (mode & SPM_ESTEP_DEFER_FOLD) != 0;
  mode &= ~SPM_ESTEP_DEFER_FOLD;
  if (mode != SPM_ESTEP_FAST && mode != SPM_ESTEP_PARITY) return Err(P, SPM_INVALID_ARGUMENT, "mode");
  if (mode == SPM_ESTEP_PARITY && (T < 1 || static_cast<uint64_t>(T) * P->V >= (1ull << 32)))
    return Err(P, SPM_INVALID_ARGUMENT, "num_threads * pieces must fit in 32 bits");
  if (n == 0) return SPM_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // Sentences per chunk; PARITY uses smaller chunks so the fold of one
  // overlaps the walks of the next.
  // The call is cut into equal chunks of at most that size: a 12.5 M-sentence
  // call used to end in a 0.5 M chunk that paid a whole chunk's fixed cost
  // (host reads, sort passes, kernel tails) for an eighth of the work.
  // (PARITY 6 M: 0.2390 vs 0.2421 s/epoch at 4 M, the c4 bench's 12.5 M-sentence
  // calls in two chunks instead of three, profiles/r05ai_estep_chunk_ab.txt.)
  uint64_t kMaxChunk = mode == SPM_ESTEP_PARITY ? (6ull << 20) : (8ull << 20);
  if (const char *e = std::getenv("SPM_HIP_ESTEP_CHUNK")) {  // A/B knob: sentences per chunk
    const unsigned long long v = std::strtoull(e, nullptr, 10);
    if (v >= 65536) kMaxChunk = v;
  }
  // The first PARITY chunk after a finalize (zero accumulators: no record
  // can be dropped, estep_threshold_kernel) is kept small; the rest of the
  // call is cut into equal chunks.  SPM_HIP_ESTEP_FIRST=0: equal chunks only.
  static const uint64_t kFirstChunk = [] {
    const char *e = std::getenv("SPM_HIP_ESTEP_FIRST");
    return e ? std::strtoull(e, nullptr, 10) : (1ull << 18);
  }();
  std::vector<uint64_t> cuts{0};
  if (mode == SPM_ESTEP_PARITY && P->fresh_acc && kFirstChunk && n > 4 * kFirstChunk) cuts.push_back(kFirstChunk);
  {
    const uint64_t b = cuts.back(), left = n - b, parts = (left + kMaxChunk - 1) / kMaxChunk;
    for (uint64_t k = 1; k <= parts; ++k) cuts.push_back(b + left * k / parts);
  }
  if (mode == SPM_ESTEP_PARITY) P->fresh_acc = false;
  if (mode == SPM_ESTEP_PARITY && !P->fold_st) {
    E_TRY(hipStreamCreateWithFlags(&P->fold_st, hipStreamNonBlocking));
    for (int k = 0; k < 2; ++k) {
      E_TRY(hipEventCreateWithFlags(&P->ev_ready[k], hipEventDisableTiming));
      E_TRY(hipEventCreateWithFlags(&P->ev_done[k], hipEventDisableTiming));
    }
  }
  int last_set = -1;
  std::vector<uint64_t> hoff(2);
  for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
    const uint64_t c0 = cuts[ci], cn = cuts[ci + 1] - c0;
    const uint64_t *off = d_off + c0;
    uint64_t lo_hi[2];
    E_TRY(hipMemcpyAsync(P->pinned, off, 8, hipMemcpyDeviceToHost, st));
    E_TRY(hipMemcpyAsync(P->pinned + 2, off + cn, 8, hipMemcpyDeviceToHost, st));
    E_TRY(hipStreamSynchronize(st));
    std::memcpy(&lo_hi[0], P->pinned, 8);
    std::memcpy(&lo_hi[1], P->pinned + 2, 8);
    // Work buffers are indexed by absolute byte offsets of the chunk.
    const uint64_t bytes_end = lo_hi[1];
    E_TRY(P->w_A.Reserve((bytes_end + 1) * 4));
    E_TRY(P->w_bp.Reserve(bytes_end + 16));
    E_TRY(P->w_Z.Reserve(cn * 4));
    E_TRY(P->w_N.Reserve(cn * 4));
    E_TRY(P->w_ntok.Reserve(cn * 4));
    E_TRY(P->w_flag.Reserve(cn * 4));
    E_TRY(P->w_status.Reserve(64));
    E_TRY(P->w_recoff.Reserve((cn + 1) * 8));
    E_TRY(hipMemsetAsync(P->w_status.ptr, 0, 64, st));
    EArgs a{};
    a.bytes = d_bytes;
    a.off = off;
    a.freq = d_freq + c0;
    a.n = cn;
    a.units = P->d_units.as<uint32_t>();
    a.values = P->d_values.as<int32_t>();
    a.scores = P->d_scores.as<float>();
    a.vscore = P->d_vscore.as<float>();
    a.uvs = P->d_uvs.as<uint2>();
    a.uvis = P->d_uvis.as<uint4>();
    a.num_units = static_cast<uint32_t>(P->trie.units.size());
    a.root_base = P->root_base;
    a.unk_score = P->unk_score;
    a.tie_mag = P->tie_mag;
    a.V = static_cast<uint32_t>(P->V);
    a.A = P->w_A.as<float>();
    a.Zlat = P->w_Z.as<float>();
    a.N = P->w_N.as<uint32_t>();
    a.ntok = P->w_ntok.as<uint32_t>();
    a.gbp = P->w_bp.as<uint8_t>();
    a.flagged = P->w_flag.as<uint32_t>();
    a.status = P->w_status.as<uint32_t>();
    a.mode = mode;
    static const int kNtRecords = [] {
      const char *e = std::getenv("SPM_HIP_ESTEP_NT");
      return e ? std::atoi(e) : 0;
    }();
    a.nt = kNtRecords;
    a.T = std::max(T, 1);
    a.index_base = index_base + c0 * index_stride;
    a.index_stride = index_stride;
    a.acc = static_cast<double *>(d_acc);
    a.acc_obj = static_cast<double *>(d_acc_obj);
    a.ntok_b = d_ntok_acc;
    a.hot_slot = P->d_hot_slot.as<int16_t>();
    a.hot_id = P->d_hot_id.as<int32_t>();
    a.all_freq_f = static_cast<float>(all_sentence_freq);
    const unsigned blocks = static_cast<unsigned>((cn + kEBlock - 1) / kEBlock);
    const bool ring_ok = P->ring_width != 0;
    if (ring_ok && !P->enc_tried && !P->enc_off.empty() && P->forward_mode != 2 &&
        (n >= kByteForwardMinSentences || P->forward_mode == 1)) {
      // A list model_from_pieces rejects (empty or duplicate piece), or one
      // its encode does not take to the byte kernel, keeps
      // estep_forward_kernel.
      P->enc_tried = true;
      if (spm_hip_model_from_pieces(reinterpret_cast<const uint8_t *>(P->enc_bytes.data()), P->enc_off.data(),
                                    P->enc_scores.data(), P->V, &P->enc) == SPM_OK &&
          !EStepByteForwardOk(P->enc)) {
        spm_hip_model_free(P->enc);
        P->enc = nullptr;
      }
    }
    ETimingMark(P, st);  // forward pass begins
    if (ring_ok && P->enc && P->forward_mode != 2) {
      // Byte-kernel E-step mode (unigram_encode.hip): the encode kernel's
      // walk (two positions per lane in flight, lagged inserts, root level
      // in LDS) with the alpha ring added.
      E_TRY(P->w_ectl.Reserve(256));
      E_TRY(hipMemsetAsync(P->w_ectl.ptr, 0, 256, st));
      EStepForwardOut eo{a.A, a.Zlat, a.N, a.ntok, a.flagged, a.status};
      const EStepKnobs &kn = Knobs();
      // (The backward kernels that read AT are the rolled ones.)
      if (kn.transposed_alpha && kn.roll && !(mode == SPM_ESTEP_PARITY && kn.stage) && P->ring_width == 16) {
        const uint64_t tiles = (cn + kEBlock - 1) / kEBlock;
        E_TRY(P->w_AT.Reserve(tiles * kATRows * kEBlock * 4));
        E_TRY(P->w_lanemap.Reserve(tiles * kEBlock));
        E_TRY(P->w_colmap.Reserve(cn * 2));
        eo.AT = P->w_AT.as<float>();
        eo.lanemap = P->w_lanemap.as<uint8_t>();
        eo.colmap = P->w_colmap.as<uint16_t>();
        a.colmap = eo.colmap;
        a.AT = eo.AT;
        a.lanemap = eo.lanemap;
      }
      const int erc = EStepByteForward(P->enc, d_bytes, off, cn, bytes_end, P->w_bp.as<uint8_t>(),
                                       P->w_ectl.as<uint32_t>(), eo, st);
      if (erc != SPM_OK) return Err(P, erc, "E-step byte forward pass launch failed");
    } else if (ring_ok) {
      // 3 waves/SIMD (measured against 2 and 4: 0.348 / 0.400 s per c4 epoch
      // vs 0.299).
      if (P->ring_width == 16) {
        hipLaunchKernelGGL((estep_forward_kernel<16, 3>), dim3(blocks), dim3(kEBlock), 0, st, a);
      } else {
        hipLaunchKernelGGL((estep_forward_kernel<32, 1>), dim3(blocks), dim3(kEBlock), 0, st, a);
      }
      E_TRY(hipGetLastError());
    }
    ETimingMark(P, st);  // forward pass ends
    if (mode == SPM_ESTEP_PARITY && !P->neg_freq_seen) {
      hipLaunchKernelGGL(estep_freq_check_kernel, dim3(std::min<unsigned>(blocks, 1024)), dim3(256), 0, st, a.freq,
                         cn, P->w_status.as<uint32_t>());
      E_TRY(hipGetLastError());
    }
    // Flag bookkeeping (+ node counts for PARITY record offsets).
    E_TRY(hipMemcpyAsync(P->pinned, P->w_status.ptr, 16, hipMemcpyDeviceToHost, st));
    E_TRY(hipStreamSynchronize(st));
    uint32_t flagged = P->pinned[0], max_nb = P->pinned[1];
    if (P->pinned[3]) P->neg_freq_seen = true;
    if (!ring_ok) {
      // Every sentence on the general path: device list + node counts.
      hipLaunchKernelGGL(estep_count_kernel, dim3((cn + 255) / 256), dim3(256), 0, st, a);
      E_TRY(hipGetLastError());
      E_TRY(hipMemcpyAsync(P->pinned, P->w_status.ptr, 8, hipMemcpyDeviceToHost, st));
      E_TRY(hipStreamSynchronize(st));
      flagged = P->pinned[0];
      max_nb = P->pinned[1];
    }
    uint64_t total_rec = 0;
    if (mode == SPM_ESTEP_PARITY) {
      // rec_off = exclusive scan of N.
      size_t tb = 0;
      hipcub::TransformInputIterator<uint64_t, ToU64E, const uint32_t *> it(a.N, ToU64E());
      E_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, it, P->w_recoff.as<uint64_t>() + 1,
                                             static_cast<int>(cn), st));
      E_TRY(P->w_tmp.Reserve(tb + 16));
      E_TRY(hipMemsetAsync(P->w_recoff.ptr, 0, 8, st));
      E_TRY(hipcub::DeviceScan::InclusiveSum(P->w_tmp.ptr, tb, it, P->w_recoff.as<uint64_t>() + 1,
                                             static_cast<int>(cn), st));
      E_TRY(hipMemcpyAsync(P->pinned + 4, P->w_recoff.as<uint64_t>() + cn, 8, hipMemcpyDeviceToHost, st));
      E_TRY(hipStreamSynchronize(st));
      std::memcpy(&total_rec, P->pinned + 4, 8);
      if (total_rec >= (1ull << 31)) return Err(P, SPM_RESOURCE_EXHAUSTED, "too many lattice nodes in a chunk");
      const uint64_t nrec = std::max<uint64_t>(total_rec, 1);
      E_TRY(P->w_keys.Reserve(nrec * 4));
      E_TRY(P->w_vals.Reserve(nrec * 8));
      E_TRY(P->w_keys2.Reserve(nrec * 4));
      a.rec_off = P->w_recoff.as<uint64_t>();
      a.keys = P->w_keys.as<uint32_t>();
      a.vals = P->w_vals.as<double>();
      // Record drop (the PARITY byte-ring backward kernel only): bounds from
      // the accumulators of the buckets this chunk touches, b = r0 (mod g).
      static const bool kNoDrop = std::getenv("SPM_HIP_ESTEP_NODROP") != nullptr;  // A/B knob
      if (ring_ok && P->ring_width == 16 && !P->neg_freq_seen && P->V < (1ull << 24) && !kNoDrop) {
        const uint64_t TT = static_cast<uint64_t>(a.T);
        uint64_t g = TT, r = a.index_stride % TT;
        while (r) {
          const uint64_t x = g % r;
          g = r;
          r = x;
        }
        E_TRY(P->w_drop.Reserve(kHot));
        E_TRY(P->w_kept.Reserve(cn * 4));
        hipLaunchKernelGGL(estep_threshold_kernel, dim3(kHot / 256), dim3(256), 0, st,
                           static_cast<const float *>(d_acc), P->V, a.T, static_cast<uint32_t>(a.index_base % g),
                           static_cast<uint32_t>(g), P->d_hot_id.as<int32_t>(),
                           static_cast<uint32_t>(std::min<uint64_t>(P->V, kHot)), P->w_drop.as<uint8_t>());
        E_TRY(hipGetLastError());
        // Sentences the kernel does not walk (general path, empty) keep all N.
        E_TRY(hipMemcpyAsync(P->w_kept.ptr, a.N, cn * 4, hipMemcpyDeviceToDevice, st));
        a.drop_exp = P->w_drop.as<uint8_t>();
        a.kept = P->w_kept.as<uint32_t>();
        // Deferred record values (SPM_HIP_ESTEP_DEFER=0: off, A/B knob).
        static const bool kDefer = [] {
          const char *e = std::getenv("SPM_HIP_ESTEP_DEFER");
          return !(e && std::atoi(e) == 0);
        }();
        if (kDefer) a.exs = reinterpret_cast<float *>(a.vals);
      }
    }
    ETimingMark(P, st);  // backward pass begins
    if (ring_ok) {
      const unsigned bblocks = std::min<unsigned>(blocks, 2048);  // LDS accumulators flushed per block
      if (P->ring_width == 16) {
        // PARITY calls: the PARITY-only lagged kernel (no FAST LDS table: 121
        // VGPRs, 14 KB LDS, 4 waves/SIMD; 0.524 -> 0.510 s/epoch at c4,
        // profiles/r02za_estep_bwd_ab.txt).  FAST keeps the batched kernel (the
        // lagged one is slower there: 0.315 vs 0.299 s/epoch, the emit work
        // sits between dependent walk steps).
        const EStepKnobs &kn = Knobs();
        if (mode == SPM_ESTEP_PARITY) {
          if (a.lanemap) {  // the forward pass wrote AT (kn.roll, !kn.stage)
            if (kn.transposed_records && a.exs) {
              const uint64_t tiles = (cn + kEBlock - 1) / kEBlock;
              E_TRY(P->w_RT.Reserve(tiles * kRTRows * kEBlock * 8));
              a.RT = P->w_RT.as<uint2>();
              a.rt_rows = kRTRows;
            }
            hipLaunchKernelGGL((estep_backward_kernel<16, 4, 42>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          } else if (kn.roll && kn.stage)
            hipLaunchKernelGGL((estep_backward_kernel<16, 4, 26>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else if (kn.roll)
            hipLaunchKernelGGL((estep_backward_kernel<16, 4, 10>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else if (kn.pair)
            hipLaunchKernelGGL((estep_backward_kernel<16, 3, 6>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else
            hipLaunchKernelGGL((estep_backward_kernel<16, 4, 3>), dim3(bblocks), dim3(kEBlock), 0, st, a);
        } else {
          if (a.lanemap)
            hipLaunchKernelGGL((estep_backward_kernel<16, 3, 40>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else if (kn.roll)
            hipLaunchKernelGGL((estep_backward_kernel<16, 3, 8>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else if (kn.pair)
            hipLaunchKernelGGL((estep_backward_kernel<16, 3, 4>), dim3(bblocks), dim3(kEBlock), 0, st, a);
          else
            hipLaunchKernelGGL((estep_backward_kernel<16, 3>), dim3(bblocks), dim3(kEBlock), 0, st, a);
        }
      } else {
        hipLaunchKernelGGL((estep_backward_kernel<32, 1>), dim3(bblocks), dim3(kEBlock), 0, st, a);
      }
      E_TRY(hipGetLastError());
    }
    ETimingMark(P, st);  // backward pass ends
    if (flagged > 0) {
      const int K = P->trie_results_size + 1;
      const uint64_t slab = EGeneralSlab(std::max<uint32_t>(max_nb, 1), K);
      uint64_t threads = std::min<uint64_t>(flagged, 16384);
      while (threads > 64 && threads * slab > (4ull << 30)) threads /= 2;
      if (threads * slab > (16ull << 30)) return Err(P, SPM_RESOURCE_EXHAUSTED, "sentence too long");
      E_TRY(P->w_scratch.Reserve(threads * slab));
      EGenArgs g{a, P->w_flag.as<uint32_t>(), P->w_status.as<uint32_t>(), P->w_scratch.as<uint8_t>(),
                 slab, std::max<uint32_t>(max_nb, 1), K, P->w_status.as<uint32_t>() + 2};
      hipLaunchKernelGGL(estep_general_kernel, dim3((threads + 63) / 64), dim3(64), 0, st, g);
      E_TRY(hipGetLastError());
    }
    if (mode == SPM_ESTEP_PARITY) {
      // Sort, segment bounds, obj records and key lists on `st`; the fold on
      // fold_st overlaps the next chunk's walks.  (Sorting on fold_st too was
      // measured slower: 0.554 vs 0.510 s/epoch — the radix sort starved of
      // CUs next to the walks took 12 ms instead of 5 per chunk.)
      const uint64_t nkeys = static_cast<uint64_t>(a.T) * P->V;
      // Dropped records: pack the kept ones densely (in order) before the sort.
      const uint32_t *sort_keys = a.keys;
      const double *sort_vals = a.vals;
      uint64_t nsort = total_rec;
      if (a.kept) {
        size_t tb = 0;
        hipcub::TransformInputIterator<uint64_t, ToU64E, const uint32_t *> it(a.kept, ToU64E());
        E_TRY(P->w_koff.Reserve((cn + 1) * 8));
        E_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, it, P->w_koff.as<uint64_t>() + 1, static_cast<int>(cn),
                                               st));
        E_TRY(P->w_tmp.Reserve(tb + 16));
        E_TRY(hipMemsetAsync(P->w_koff.ptr, 0, 8, st));
        E_TRY(hipcub::DeviceScan::InclusiveSum(P->w_tmp.ptr, tb, it, P->w_koff.as<uint64_t>() + 1,
                                               static_cast<int>(cn), st));
        E_TRY(hipMemcpyAsync(P->pinned + 8, P->w_koff.as<uint64_t>() + cn, 8, hipMemcpyDeviceToHost, st));
        E_TRY(hipStreamSynchronize(st));
        std::memcpy(&nsort, P->pinned + 8, 8);
        if (nsort > total_rec) return Err(P, SPM_INTERNAL, "E-step record drop: kept more records than written");
        if (nsort < total_rec || a.exs) {
          E_TRY(P->w_ckeys.Reserve(std::max<uint64_t>(nsort, 1) * 4));
          E_TRY(P->w_cvals.Reserve(std::max<uint64_t>(nsort, 1) * 8));
          hipLaunchKernelGGL(estep_compact_records_kernel, dim3(static_cast<unsigned>((cn + 255) / 256)), dim3(256),
                             0, st, cn, a.rec_off, a.N, a.kept, P->w_koff.as<uint64_t>(), a.keys, a.vals, a.exs,
                             a.freq, P->w_ckeys.as<uint32_t>(), P->w_cvals.as<double>(), a.RT,
                             P->w_colmap.as<uint16_t>(), a.rt_rows);
          E_TRY(hipGetLastError());
          sort_keys = P->w_ckeys.as<uint32_t>();
          sort_vals = P->w_cvals.as<double>();
        }
      }
      P->rec_total += total_rec;
      P->rec_kept += nsort;
      const int set = static_cast<int>(P->fold_chunks++ & 1);
      // The fold two chunks back read this set: wait for it before reuse
      // (and on the host before a buffer of the set has to grow).
      if (P->ev_used[set]) {
        if (P->w_svals[set].cap < std::max<uint64_t>(nsort, 1) * 8 || P->w_sobjq[set].cap < cn * 8)
          E_TRY(hipEventSynchronize(P->ev_done[set]));
        E_TRY(hipStreamWaitEvent(st, P->ev_done[set], 0));
      }
      E_TRY(P->w_svals[set].Reserve(std::max<uint64_t>(nsort, 1) * 8));
      E_TRY(P->w_sseg[set].Reserve((nkeys + 1) * 8));
      E_TRY(P->w_sobjq[set].Reserve(cn * 8));
      E_TRY(P->w_heavy[set].Reserve(std::max<uint64_t>(nkeys, 1) * 4));
      E_TRY(P->w_light[set].Reserve(std::max<uint64_t>(nkeys, 1) * 4));
      E_TRY(P->w_cls[set].Reserve(8));
      double *svals = P->w_svals[set].as<double>();
      uint64_t *sseg = P->w_sseg[set].as<uint64_t>();
      double *sobjq = P->w_sobjq[set].as<double>();
      uint32_t *cls = P->w_cls[set].as<uint32_t>();
      int end_bit = 1;
      while ((1ull << end_bit) < nkeys) ++end_bit;
      // Stable onesweep radix sort with 10-bit digits: the keys have 19 bits
      // (T = 16, V = 32k), so two passes instead of hipcub's three 8-bit ones
      // (150 M records: 2.97 vs 4.62 ms, same permutation,
      // profiles/r03j_sort_ab.txt, tools/sort_ab.hip).
      size_t tb = 0;
      E_TRY(rocprim::radix_sort_pairs<RecordSortConfig>(nullptr, tb, sort_keys, P->w_keys2.as<uint32_t>(),
                                                        sort_vals, svals, nsort, 0, end_bit, st));
      E_TRY(P->w_tmp.Reserve(tb + 16));
      if (nsort)
        E_TRY(rocprim::radix_sort_pairs<RecordSortConfig>(P->w_tmp.ptr, tb, sort_keys, P->w_keys2.as<uint32_t>(),
                                                          sort_vals, svals, nsort, 0, end_bit, st));
      hipLaunchKernelGGL(estep_seg_bounds_kernel, dim3((nkeys + 1 + 255) / 256), dim3(256), 0, st,
                         P->w_keys2.as<uint32_t>(), nsort, nkeys, sseg);
      E_TRY(hipGetLastError());
      hipLaunchKernelGGL(estep_objq_kernel, dim3(static_cast<unsigned>((cn + 255) / 256)), dim3(256), 0, st, a,
                         sobjq);
      E_TRY(hipGetLastError());
      // Heavy / light key lists; the fold reads their sizes on the device.
      E_TRY(hipMemsetAsync(cls, 0, 8, st));
      hipLaunchKernelGGL(estep_classify_kernel, dim3(static_cast<unsigned>((nkeys + 255) / 256)), dim3(256), 0, st,
                         sseg, nkeys, P->w_heavy[set].as<uint32_t>(), P->w_light[set].as<uint32_t>(), cls);
      E_TRY(hipGetLastError());
      // Fold on the side stream, after everything queued on `st` so far: the
      // T obj chains + kFoldBlocks grid-stride wavefronts over the key lists.
      E_TRY(hipEventRecord(P->ev_ready[set], st));
      E_TRY(hipStreamWaitEvent(P->fold_st, P->ev_ready[set], 0));
      // 4096 single-wave blocks (grid-stride): the fold then leaves more of
      // the CUs to the next chunk's walks it overlaps; c4 PARITY 0.413 s/epoch
      // vs 0.422 with 16384 and 0.430 with 1024 (profiles/r03t_fold_blocks_ab.txt).
      constexpr unsigned kFoldBlocks = 4096;
      // 4 records per lane and window (66 VGPRs, 7 waves/SIMD): the fold's
      // waves then take less of the register file from the walks they run
      // beside; c4 PARITY 0.4245 -> 0.4199 s/epoch vs 16 (248 VGPRs), 8 is
      // 0.4323 (profiles/r03za_fold_ab.txt).
      hipLaunchKernelGGL(estep_fold_kernel<4>, dim3(static_cast<unsigned>(a.T) + kFoldBlocks), dim3(64), 0,
                         P->fold_st, a, sobjq, static_cast<float *>(d_acc_obj), sseg, svals,
                         static_cast<float *>(d_acc), P->w_heavy[set].as<uint32_t>(),
                         P->w_light[set].as<uint32_t>(), cls);
      E_TRY(hipGetLastError());
      E_TRY(hipEventRecord(P->ev_done[set], P->fold_st));
      P->ev_used[set] = true;
      last_set = set;
    }
    if (flagged > 0) {
      E_TRY(hipMemcpyAsync(P->pinned + 6, P->w_status.as<uint32_t>() + 2, 4, hipMemcpyDeviceToHost, st));
      E_TRY(hipStreamSynchronize(st));
      if (P->pinned[6]) return Err(P, SPM_INTERNAL, "general E-step path: scratch overflow");
    }
  }
  // The caller's stream sees the accumulators after the last fold (unless
  // deferred: spm_hip_estep_sync / finalize make that wait).
  if (last_set >= 0 && !defer) E_TRY(hipStreamWaitEvent(st, P->ev_done[last_set], 0));
  return SPM_OK;
}

int spm_hip_estep_sync(spm_hip_pieces *P, void *stream) {
  using namespace spm_amd;
  if (!P) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  // Folds run in order on fold_st: the later of the two sets' events covers
  // every fold enqueued so far; waiting on both is the same.
  for (int k = 0; k < 2; ++k)
    if (P->ev_used[k]) E_TRY(hipStreamWaitEvent(st, P->ev_done[k], 0));
  return SPM_OK;
}

int spm_hip_estep_finalize(spm_hip_pieces *P, int mode, int T, const void *d_acc, const void *d_acc_obj,
                           const int64_t *d_ntok_acc, float *d_expected, float *d_obj, int64_t *d_ntok,
                           void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_estep_finalize");
  using namespace spm_amd;
  if (!P) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int src = spm_hip_estep_sync(P, stream);  // deferred folds first
  if (src != SPM_OK) return src;
  P->fresh_acc = true;  // the caller's next E-step starts from zero accumulators
  hipLaunchKernelGGL(estep_finalize_kernel, dim3((P->V + 255) / 256), dim3(256), 0, st, mode,
                     std::max(T, 1), P->V, static_cast<const double *>(d_acc),
                     static_cast<const double *>(d_acc_obj), static_cast<const float *>(d_acc),
                     static_cast<const float *>(d_acc_obj), d_ntok_acc, d_expected, d_obj, d_ntok);
  E_TRY(hipGetLastError());
  return SPM_OK;
}

int spm_hip_estep(spm_hip_pieces *P, const uint8_t *d_bytes, const uint64_t *d_off,
                  const int64_t *d_freq, uint64_t n, int64_t all_sentence_freq, int mode, int T,
                  float *d_expected, float *d_obj, int64_t *d_ntok, void *stream) {
  using namespace spm_amd;
  if (!P) return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int TT = mode == SPM_ESTEP_PARITY ? std::max(T, 1) : 1;
  const uint64_t acc_bytes = mode == SPM_ESTEP_FAST ? P->V * 8 : static_cast<uint64_t>(TT) * P->V * 4;
  const uint64_t obj_bytes = mode == SPM_ESTEP_FAST ? 8 : static_cast<uint64_t>(TT) * 4;
  E_TRY(P->w_red.Reserve(acc_bytes + 256 + obj_bytes + TT * 8ull));
  char *base = P->w_red.as<char>();
  void *acc = base;
  void *acc_obj = base + ((acc_bytes + 255) / 256) * 256;
  int64_t *ntok_acc = reinterpret_cast<int64_t *>(static_cast<char *>(acc_obj) + ((obj_bytes + 7) / 8) * 8);
  E_TRY(hipMemsetAsync(base, 0, P->w_red.cap, st));
  int rc = spm_hip_estep_accumulate(P, d_bytes, d_off, d_freq, n, all_sentence_freq, mode, TT, 0, 1,
                                    acc, acc_obj, ntok_acc, stream);
  if (rc != SPM_OK) return rc;
  return spm_hip_estep_finalize(P, mode, TT, acc, acc_obj, ntok_acc, d_expected, d_obj, d_ntok, stream);
}


int spm_hip_prune_nbest(spm_hip_pieces *P, const uint8_t *d_piece_bytes, const uint64_t *d_piece_off,
                        uint8_t *d_keep, int32_t *d_alt, const uint64_t *d_alt_off, uint32_t *d_alt_n,
                        uint32_t max_piece_bytes, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_prune_nbest");
  using namespace spm_amd;
  if (!P || !d_piece_bytes || !d_piece_off || !d_keep || !d_alt || !d_alt_off || !d_alt_n)
    return SPM_INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> lock(P->mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  constexpr uint32_t kMaxHyps = 4096;
  const int K = P->trie_results_size + 1;
  const uint32_t max_nb = std::max<uint32_t>(max_piece_bytes, 1);
  const uint64_t slab = NBestSlab(max_nb, K, kMaxHyps);
  uint64_t threads = std::min<uint64_t>(std::max<uint64_t>(P->V, 1), 16384);
  while (threads > 64 && threads * slab > (1ull << 30)) threads /= 2;
  E_TRY(P->w_scratch.Reserve(threads * slab));
  NBestArgs g{d_piece_bytes, d_piece_off, P->V, P->d_units.as<uint32_t>(), P->d_values.as<int32_t>(),
              P->d_scores.as<float>(), P->root_base, P->unk_score, P->w_scratch.as<uint8_t>(), slab,
              max_nb, K, kMaxHyps, d_keep, d_alt, d_alt_off, d_alt_n};
  hipLaunchKernelGGL(prune_nbest_kernel, dim3(static_cast<unsigned>((threads + 63) / 64)), dim3(64), 0, st, g);
  E_TRY(hipGetLastError());
  return SPM_OK;
}

}  // extern "C"
