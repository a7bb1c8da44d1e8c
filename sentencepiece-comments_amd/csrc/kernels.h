// Kernel launch interfaces (internal; the public boundary is include/spm_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_types.h"
#include "normalize_device.h"

namespace spm_amd {

// Words of the per-call status block (zeroed by the host at the start of
// every encode call, stream-ordered).
enum : int {
  kStFlagged = 0,   // sentences the fast kernel handed to the general kernel
  kStMaxNb = 1,     // longest flagged sentence (bytes)
  kStError = 2,     // bit 0: a flagged sentence outgrew the device general path
  kStTicket = 3,    // tile tickets of the fast kernel
  kStOverflow = 4,  // flagged sentences longer than the general kernel's lane slab
  kStScanTicket = 5,// tile tickets of the fix-up scan
  kStCoopRest = 6,  // flagged sentences the cooperative kernel handed to the general kernel
  kStCoopQueue = 7, // the cooperative list kernel's work queue (next list entry)
  kStCoopLong = 8,  // coop partition: long sentences (taken first)
  kStCoopShort = 9, // coop partition: the others
  kStWords = 16
};

// Token-offset entry of a flagged sentence (fast kernel output): bit 63 set,
// low bits the (exclusive) offset; the fix-up kernels strip it.
constexpr uint64_t kTokFlag = 1ull << 63;

// Unigram encode of one batch (unigram_encode.hip).  The fast kernel writes
// each tile's (256 sentences) tokens densely into slot[off[256 t] ..] with
// tile-local token offsets in tok_off and the tile's count in tile_count[t];
// LaunchTileCompact scans the counts and places every tile, so ids[] /
// piece_len[] / tok_off[] are then final for every sentence it handled.  A
// sentence it cannot handle exactly is appended to `flagged`, gets zero
// tokens and its tok_off[i + 1] entry carries kTokFlag; the general kernel
// and the fix-up kernels (all device-guarded by the flagged count, so they
// are no-ops in the common case) then splice its tokens in.
struct UnigramLaunch {
  const uint8_t *bytes;
  const uint64_t *off;
  uint64_t n;
  uint64_t capacity;         // caller's bound on off[n] (every scratch buffer is sized by it)
  const uint32_t *units;     // byte kernel: (0xFF-padded unit, node score) pairs
  const uint32_t *gen_units; // the plain double array (general kernel)
  const int32_t *values;
  const float *scores;
  uint32_t num_units;
  UnigramParams p;
  int32_t *ids;              // dense output (written by the fix-up / tile compaction)
  uint32_t *len;             // nullable
  uint64_t *tok_off;         // n + 1
  uint8_t *bp;               // back-pointer scratch: >= offsets[n] + 16 bytes
  uint32_t *flagged;         // n entries
  uint32_t *status;          // kStWords
  uint64_t *tile_count;      // FastTiles(n) tile token counts
  uint64_t corrupt_bp;       // debug: zero this sentence's EOS back-pointer (~0: off)
  const uint32_t *chain;     // caller's status word (nullable): skip everything if non-zero
  int32_t *slot_ids;         // tile-dense token slots (capacity entries)
  uint32_t *slot_len;        // nullable
  uint32_t *bpn;             // kWide: trie unit per byte position (capacity + 16 entries)
  // Single-tile host calls (EncodeHostSmall): the block first zeroes words
  // [0, stage_zero) of stage_dst (the status block) and copies words
  // [stage_zero, stage_words) of the call's input image (offsets, bytes)
  // from pinned host memory, and at its end publishes the status words to
  // host_pub[1..kStWords] and then pub_seq to host_pub[0].
  const uint32_t *stage_src;
  uint32_t *stage_dst;
  uint32_t stage_zero;
  uint32_t stage_words;
  uint32_t *host_pub;
  uint32_t pub_seq;
  // Wide / char kernels: sentences of >= coop_min_nb bytes (0: none) are
  // flagged without a walk, for the wave-cooperative kernel (coop_encode.hip).
  uint32_t coop_min_nb;
};

enum class UnigramKernel : int { kGeneralOnly = 0, kByte = 1, kChar = 2, kWide = 3 };

// The unigram trainer E-step's forward pass in the byte kernel (estep mode):
// per sentence Z (alpha of EOS), N (lattice nodes), ntok (Viterbi().size(),
// kNone when flagged to the general E-step kernel), alpha at every char start
// at A[offset], flagged list + fstatus[0] count / [1] max flagged bytes.
struct EStepForwardOut {
  float *A;
  float *Z;
  uint32_t *N;
  uint32_t *ntok;
  uint32_t *flagged;
  uint32_t *fstatus;
  // Tile-transposed alpha (null: A only).  Tile t = sentences [256t, 256t +
  // 256); the pass's lane l of tile t walks sentence 256t + lanemap[256t + l]
  // (its length sort) and writes alpha of byte position p < kATRows to
  // AT[(t * kATRows + p) * 256 + l], so a wave's 64 lanes store one 256-byte
  // run per position instead of 64 scattered dwords; positions >= kATRows go
  // to A.  colmap[i] = the lane of sentence i (the backward pass sets 0xFFFF
  // for a general-path sentence).  The backward pass reads AT with the same
  // lane assignment.
  float *AT = nullptr;
  uint8_t *lanemap = nullptr;
  uint16_t *colmap = nullptr;
};
constexpr uint32_t kATRows = 64;

inline uint64_t FastTiles(uint64_t n) { return (n + 255) / 256; }
hipError_t LaunchUnigramEStepForward(const UnigramLaunch &l, const EStepForwardOut &e, hipStream_t st);
}  // namespace spm_amd
struct spm_hip_model;
namespace spm_amd {
// spm_hip_api.cc: the E-step forward pass through a TrainerModel's byte
// kernel (ok: the model encodes with the byte kernel, W = 16).
bool EStepByteForwardOk(const spm_hip_model *m);
int EStepByteForward(spm_hip_model *m, const uint8_t *bytes, const uint64_t *off, uint64_t n, uint64_t bytes_end,
                     uint8_t *bp, uint32_t *ctl, const EStepForwardOut &e, hipStream_t st);
constexpr uint64_t kScanTiles = 1024;  // look-back tiles of the fix-up scan

// The fast kernel for the model's kernel kind: kByte (ring W = 16, the c2
// kernel) or kChar (W = 16/32/64).
hipError_t LaunchUnigramFast(UnigramKernel kind, int ring_width, const UnigramLaunch &l, hipStream_t st);

// General kernel (the reference lattice literally) over a list of sentences:
// list == nullptr means all of them (count ignored, list_n used); otherwise
// *count entries of list.  Sentences longer than max_nb go to ovf_list /
// *ovf_count when ovf_list is set, else set bit 0 of *error and get 0 tokens.
// Tokens are written right-aligned in the sentence's own byte range of
// slot_ids / slot_len, counts to ntok[i].
struct GeneralLaunch {
  const uint32_t *list;
  const uint32_t *count;
  uint64_t list_n;
  uint8_t *scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;
  uint32_t threads;
  uint32_t *ovf_list;
  uint32_t *ovf_count;
  uint32_t *error;
  int32_t *slot_ids;
  uint32_t *slot_len;
  uint32_t *ntok;
};
hipError_t LaunchUnigramGeneral(const UnigramLaunch &l, const GeneralLaunch &g, hipStream_t st);

// Wave-cooperative encode (coop_encode.hip): one sentence per wavefront over a
// device list (or all list_n sentences when list is null).  Output contract of
// the general kernel: tokens right-aligned in slot_ids / slot_len of the
// sentence's byte range, ntok[i]; sentences it does not take are appended to
// rest / *rest_count.  Scratch rows by char ordinal (see slab_chars below):
// 16 + 32 bytes per char.
constexpr int kCoopSlots = 8;
struct CoopArgs {
  const uint8_t *bytes;
  const uint64_t *off;
  const uint32_t *uvs;     // (0xFF-padded unit, node score) pairs (NaN: no usable node)
  const int32_t *values;
  uint32_t num_units;
  UnigramParams p;
  const uint32_t *list;
  const uint32_t *count;
  uint64_t list_n;
  int32_t *slot_ids;
  uint32_t *slot_len;      // nullable
  uint32_t *ntok;
  uint32_t *rest;
  uint32_t *rest_count;
  // Scratch by CHAR START ordinal of the sentence: kCoopSlots chosen lnodes
  // (length | slot << 7 | chars << 10) and kCoopSlots trie nodes per char.
  // slab_chars = 0: the sentence's rows start at its byte offset b0 (a
  // sentence has at most nb chars: capacity = the call's bytes); otherwise
  // wave w (blockIdx * 4 + wave) owns rows [w * slab_chars, (w + 1) *
  // slab_chars) and a sentence of more chars goes to the general kernel.
  uint16_t *pv_scratch;    // 16-byte aligned
  uint32_t *nd_scratch;    // 16-byte aligned
  uint32_t max_len;        // longest node in bytes (pieces, and 4 for UNK); <= 56
  const uint32_t *chain;   // asynchronous chain status (nullable)
  uint64_t *prof;          // debug (SPM_HIP_COOP_PROF): 8 cycle / size counters, nullable
  uint64_t slab_chars;     // 0: rows at b0; else per-wave slabs of this many chars
  // List kernel work queue (nullable: static grid stride): waves take list
  // entries one at a time from *queue; with `part` the k-th entry is
  // part[k] for k < *part_long (the long sentences, first), else
  // part[part_n - 1 - (k - *part_long)].
  uint32_t *queue;
  const uint32_t *part;
  const uint32_t *part_long;
  uint64_t part_n;
};
// Sentences of at least this many bytes start first (the longest lines
// decide the list kernel's tail).
constexpr uint32_t kCoopLongNb = 2048;
hipError_t LaunchCoopPartition(const uint32_t *list, const uint32_t *count, const uint64_t *off, uint64_t n,
                               uint32_t *part, uint32_t *n_long, uint32_t *n_short, hipStream_t st);
// Per-wave slab of the list kernel (coop_list_kernel) and its grid cap (3
// blocks of 4 waves are resident per CU: more blocks only queue).
constexpr uint64_t kCoopSlabChars = 16384;
constexpr uint32_t kCoopMaxBlocks = 768;
hipError_t LaunchCoopEncode(const CoopArgs &a, uint32_t max_blocks, hipStream_t st);
inline uint32_t CoopBlocks(uint64_t n, uint32_t max_blocks = kCoopMaxBlocks) {
  const uint64_t b = (n + 3) / 4;
  return static_cast<uint32_t>(b < max_blocks ? b : max_blocks);
}

// One-block host call of <= kCoopSmallMax sentences (EncodeHostSmall): input
// image [offsets | bytes] staged from pinned host memory (CoopCall::
// stage_words words to stage_dst; a.off = the staged offsets, a.bytes = the
// image, the bytes at CoopCall::in_at), outputs (tok, ids, len) and the
// publication (host_pub[1] = 0 ok / 1 re-run on the lane kernels, then
// host_pub[0] = pub_seq) written into pinned host memory.
constexpr uint32_t kCoopSmallMax = 16;
struct CoopSmallArgs {
  CoopArgs a;
  const uint32_t *stage_src;
  uint32_t *stage_dst;
};
struct CoopCall;
hipError_t LaunchCoopSmall(const CoopSmallArgs &s, const CoopCall &c, hipStream_t st);
// Small raw-line calls (coop_encode.hip coop_raw_kernel): one block, n <=
// kCoopSmallMax raw lines; each wave normalizes a line (NormalizePrefix of
// 64 positions at a time, the state machine on one lane), encodes it with
// CoopEncodeSentence and merges its unknown runs; outputs and the completion
// word go to host memory.  The staged image is [raw offsets | raw bytes];
// line i's normalized bytes go to a.bytes + 4 raw_off[i] + 8 i (capacity
// 4 len + 8).
// (Per call, CoopCall: n, stage_words, in_at = the raw bytes' offset in the
// staged image, ids_cap, tok = out_off (host, n + 1), ids (host), host_pub.)
struct CoopRawArgs {
  CoopArgs a;
  NormTables t;
  const uint32_t *stage_src;
  uint32_t *stage_dst;
  const uint8_t *types;      // piece type bits (epilogue.h), num_types entries
  int32_t num_types;
};
hipError_t LaunchCoopRaw(const CoopRawArgs &s, const CoopCall &c, hipStream_t st);

// What varies between the one-block small calls (coop_small_kernel /
// coop_raw_kernel / the service kernel): sizes, the input's place in the
// staged image and the host-memory outputs.
struct CoopCall {
  uint32_t n;
  uint32_t stage_words;
  uint32_t pub_seq;
  uint32_t pad;
  uint64_t in_at;       // small: staged byte offset of the sentence bytes (b0 = in_at + off[i]); raw: of the raw bytes
  uint64_t ids_cap;     // raw: capacity of ids
  uint64_t *tok;        // small: token offsets; raw: out_off (n + 1)
  int32_t *ids;
  uint32_t *len;        // small: piece byte lengths (nullable)
  uint32_t *host_pub;   // [0] sequence, [1] 0 = done, 1 = not taken
};
// Resident service kernel for small calls (coop_service_kernel): one block
// polls `box` in pinned coherent host memory; the host writes `call` and
// then `seq` = (sequence & 0x3FFFFFFF) | kind << 30 (kind 1 = normalized
// batch with `small`'s tables, 2 = raw lines with `raw`'s); the block serves
// it exactly as coop_small_kernel / coop_raw_kernel would and publishes the
// result the same way.  It exits when `stop` is set or after idle_ticks
// wall-clock ticks without a request (then alive = 0).
struct CoopServiceBox {
  uint32_t seq;
  uint32_t stop;
  uint32_t alive;  // device: 1 from start to exit
  uint32_t served;  // device: requests served by this launch
  CoopCall call;
  // device (diagnostics, SPM_HIP_SERVICE_PROF): wall-clock ticks summed over
  // the served requests: seq seen -> call copied, -> result published.
  uint64_t ticks_copy, ticks_busy;
};
struct CoopServiceArgs {
  CoopSmallArgs small;
  CoopRawArgs raw;
  CoopServiceBox *box;
  uint32_t last;        // the box's seq at launch (a different seq is a request)
  uint64_t idle_ticks;
};
hipError_t LaunchCoopService(const CoopServiceArgs &s, hipStream_t st);
uint64_t UnigramGeneralSlabBytes(uint32_t max_nb, int trie_results_size);

// Fix-up chain after the general kernel (all no-ops when status[kStFlagged]
// is 0): fast-path tokens move to their sentences' right-aligned slots, the
// counts are re-scanned into tok_off, and every sentence is compacted back
// into ids/len.  Writes the call's final status code to out_status (nullable).
struct FixupLaunch {
  const uint64_t *off;
  uint64_t n;
  int32_t *ids;
  uint32_t *len;
  uint64_t *tok_off;
  int32_t *slot_ids;
  uint32_t *slot_len;
  const uint32_t *ntok;      // general kernel counts (flagged sentences)
  uint32_t *cnt;             // n scratch
  uint32_t *status;
  uint64_t *scan_desc;       // kScanTiles, zeroed
  uint32_t *out_status;
};
hipError_t LaunchEncodeFixup(const FixupLaunch &f, hipStream_t st);

// status[0] = code unless it is already non-zero (first error wins), on st.
hipError_t LaunchStatusSetFirst(uint32_t *status, uint32_t code, hipStream_t st);

// After the fast kernel: tile t's tokens sit densely at slot[off[256 t]],
// tile_count[t] = their count, tok_off holds tile-local inclusive offsets.
// Scans the tile counts (tile_prefix: tiles + 1 entries) and moves every
// tile to its final place with coalesced copies, rebasing tok_off.
hipError_t LaunchTileCompact(const uint64_t *off, uint64_t n, const uint64_t *tile_count, uint64_t *tile_prefix,
                             const int32_t *slot_ids, const uint32_t *slot_len, int32_t *ids, uint32_t *len,
                             uint64_t *tok_off, void *scan_tmp, size_t *scan_tmp_bytes, const uint32_t *status,
                             hipStream_t st);

// Dense CSR output from right-aligned slots (general-only and BPE paths):
// tok_off = exclusive scan of ntok; sentence i's tokens come from
// slot[off[i+1] - ntok[i]].  Skipped when status[kStError] bit 1 (the batch
// exceeded the caller's capacity) is set.
hipError_t LaunchCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok, const int32_t *slot_ids,
                         const uint32_t *slot_len, int32_t *ids, uint32_t *piece_len, uint64_t *tok_off,
                         void *scan_tmp, size_t *scan_tmp_bytes, const uint32_t *status, uint32_t *out_status,
                         hipStream_t st);

}  // namespace spm_amd
