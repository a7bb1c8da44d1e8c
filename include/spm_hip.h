/*
 * spm_hip.h — C-ABI of the MI355X-native SentencePiece encode / E-step engine.
 *
 * This is the drop-in boundary for the hot path of SentencePiece v0.1.82
 * (ycaptain/SentencePiece-comments).  Every entry point is plain C: pointers,
 * sizes and int status codes; no torch or C++ types.  Status codes are the
 * values of util::error::Code (reference src/sentencepiece_processor.h:101-119);
 * HIP failures map to SPM_INTERNAL.  No entry point aborts or throws.
 *
 * Reference interfaces replaced:
 *   spm_hip_model_load   ModelFactory::Create (src/model_factory.cc:26-47) +
 *                        unigram::Model::Model (src/unigram_model.cc:677-695) /
 *                        bpe::Model::Model (src/bpe_model.cc:26-31) +
 *                        ModelInterface::InitializePieces (src/model_interface.cc:101-144)
 *   spm_hip_encode_batch ModelInterface::Encode(normalized) (src/model_interface.h:117),
 *                        batched over sentences: unigram::Model::Encode
 *                        (src/unigram_model.cc:705-720) and bpe::Model::Encode
 *                        (src/bpe_model.cc:37-199)
 *   spm_hip_finalize_ids SentencePieceProcessor::PopulateSentencePieceText +
 *                        ApplyExtraOptions (src/sentencepiece_processor.cc:488-551,
 *                        :945-979), id part
 *   spm_hip_estep        unigram::Trainer::RunEStep (src/unigram_model_trainer.cc:237-287)
 *   spm_hip_seed_mine    unigram::Trainer::MakeSeedSentencePieces
 *                        (src/unigram_model_trainer.cc:124-225) + esaxx
 *                        (third_party/esaxx/esa.hxx:37-122)
 */
#ifndef SPM_HIP_H_
#define SPM_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version of this ABI (struct layouts and entry-point signatures).  Structs
 * such as spm_hip_model_info may change between versions; callers built
 * against another version must not use them (check spm_hip_abi_version()). */
#define SPM_HIP_ABI_VERSION 3
int spm_hip_abi_version(void);

/* util::error::Code (sentencepiece_processor.h:101-119). */
enum spm_status {
  SPM_OK = 0,
  SPM_CANCELLED = 1,
  SPM_UNKNOWN = 2,
  SPM_INVALID_ARGUMENT = 3,
  SPM_NOT_FOUND = 5,
  SPM_PERMISSION_DENIED = 7,
  SPM_RESOURCE_EXHAUSTED = 8,
  SPM_FAILED_PRECONDITION = 9,
  SPM_OUT_OF_RANGE = 11,
  SPM_UNIMPLEMENTED = 12,
  SPM_INTERNAL = 13
};

/* TrainerSpec::ModelType (sentencepiece_model.proto:29-34). */
enum spm_model_type { SPM_UNIGRAM = 1, SPM_BPE = 2, SPM_WORD = 3, SPM_CHAR = 4 };

typedef struct spm_hip_model spm_hip_model;

typedef struct spm_hip_model_info {
  int32_t model_type;       /* spm_model_type */
  int32_t piece_size;       /* ModelProto.pieces_size() */
  int32_t unk_id;           /* index of the UNKNOWN piece */
  int32_t max_piece_chars;  /* longest matchable piece, in UTF-8 chars */
  int32_t trie_results_size;/* unigram: max prefix matches per position */
  int32_t trie_units;       /* device double-array size (units) */
  float min_score;          /* unigram: min over NORMAL scores */
  float max_score;          /* unigram: max(FLT_MIN, NORMAL scores) */
  int32_t ring_width;       /* unigram fast kernel ring W (16/32/64; > longest
                               piece in bytes), 0 = general kernel only */
  int32_t fast_variant;     /* unigram encode kernel: 1 byte-position kernel
                               (W = 16), 2 char-position kernel, 3 wide-char
                               kernel (ring of 16 chars), 0 general only */
} spm_hip_model_info;

/* Counters of the last encode call (host-visible after it returns). */
typedef struct spm_hip_encode_stats {
  uint64_t sentences;
  uint64_t tokens;
  uint64_t general_path;    /* sentences re-run by the exact general kernel */
  float fast_kernel_ms;     /* HIP-event time of the fast kernel launch (0 if
                               timing is off, see spm_hip_model_set_timing) */
  float general_kernel_ms;  /* same for the general kernel */
  uint64_t coop_rest;       /* of general_path: sentences the wave-cooperative
                               kernel took first and handed on to the general
                               kernel (host batch calls) */
} spm_hip_encode_stats;

/* Parses a serialized ModelProto, validates it like InitializePieces and
 * uploads the device-resident tables (trie, scores, piece types) to the
 * current HIP device.  *out is NULL on failure. */
int spm_hip_model_load(const void *model_proto, size_t len, spm_hip_model **out);
/* Same parsing/validation and host tables, no device work (CPU-only use:
 * normalization, info).  Encode calls on such a handle return
 * SPM_FAILED_PRECONDITION. */
int spm_hip_model_load_host_only(const void *model_proto, size_t len, spm_hip_model **out);
void spm_hip_model_free(spm_hip_model *model);
/* Unigram model over a bare piece list with the trainer's TrainerModel
 * semantics (unigram_model_trainer.cc:97-119, unigram_model_trainer.h:39-89):
 * all pieces NORMAL, value = list index, unk_id 0, UNK score min - 10.  Used
 * by the pruning step's Viterbi (PruneSentencePieces :377-421) through
 * spm_hip_encode_batch.  HOST pointers. */
int spm_hip_model_from_pieces(const uint8_t *piece_bytes, const uint64_t *piece_offsets,
                              const float *scores, uint64_t num_pieces, spm_hip_model **out);
int spm_hip_model_get_info(const spm_hip_model *model, spm_hip_model_info *info);

/* Batched ModelInterface::Encode over normalized sentences, DEVICE pointers.
 *   d_norm_bytes   : concatenated normalized UTF-8 bytes (CSR values)
 *   d_offsets      : uint64[n+1] byte offsets of each sentence
 *   d_ids          : int32 output, capacity >= offsets[n] (one token per byte
 *                    is the upper bound)
 *   d_piece_len    : optional (may be NULL) uint32 byte length of each piece;
 *                    pieces are views into the input, in order
 *   d_tok_offsets  : uint64[n+1] output CSR offsets into d_ids
 *   stream         : hipStream_t (NULL = default stream)
 * BLOCKING: reads offsets[n], enqueues the work on `stream`, waits for it and
 * returns the status the reference's Encode would (util::Status).  Empty
 * sentences yield zero tokens (unigram_model.cc:706-708).  Pipelines use
 * spm_hip_encode_batch_async. */
int spm_hip_encode_batch(spm_hip_model *model, const uint8_t *d_norm_bytes,
                         const uint64_t *d_offsets, uint64_t n, int32_t *d_ids,
                         uint32_t *d_piece_len, uint64_t *d_tok_offsets, void *stream);

/* Same encode as a pure stream call: no host synchronization, all work
 * enqueued on `stream`.
 *   capacity : the caller's bound on offsets[n] (d_ids and d_piece_len hold
 *              at least that many entries); every scratch buffer is sized by
 *              it, so the offsets are never read back.
 *   d_status : DEVICE uint32 status word, zeroed by the caller before a chain
 *              of asynchronous calls.  Every kernel of these calls does
 *              nothing once it is non-zero, and the first failure stores its
 *              spm_status code (first error wins): RESOURCE_EXHAUSTED when
 *              offsets[n] > capacity, or when a sentence the fast kernel
 *              handed to the exact general kernel is longer than its device
 *              scratch (> 256 KiB; spm_hip_encode_batch handles those).
 * The return value reports argument and enqueue errors only.  Models whose
 * encode needs host-sized scratch (unigram pieces of >= 64 bytes, BPE with
 * user-defined symbols, force_general) fall back to the blocking path. */
int spm_hip_encode_batch_async(spm_hip_model *model, const uint8_t *d_norm_bytes,
                               const uint64_t *d_offsets, uint64_t n, uint64_t capacity, int32_t *d_ids,
                               uint32_t *d_piece_len, uint64_t *d_tok_offsets, uint32_t *d_status,
                               void *stream);

/* Same contract with HOST buffers; stages through pooled device buffers and
 * returns after the results are copied back. */
int spm_hip_encode_batch_host(spm_hip_model *model, const uint8_t *norm_bytes,
                              const uint64_t *offsets, uint64_t n, int32_t *ids,
                              uint32_t *piece_len, uint64_t *tok_offsets);

/* Normalizer::Normalize (normalizer.cc:88-211) on host threads, batched:
 * raw CSR lines in, normalized CSR out.  out capacity: 3*in_off[n] + 3*n
 * bytes.  norm_to_orig is not produced.  num_threads <= 0 → hardware
 * concurrency. */
int spm_hip_normalize_batch(const spm_hip_model *model, const uint8_t *in, const uint64_t *in_off,
                            uint64_t n, uint8_t *out, uint64_t *out_off, int num_threads);

/* Normalizer::Normalize (normalizer.cc:88-211, NormalizePrefix :231-300 over
 * the model's precompiled charsmap and user-defined PrefixMatcher) on the
 * device, batched.  DEVICE pointers: raw CSR in (d_in, d_in_off[n+1]),
 * normalized CSR out (d_out, d_out_off[n+1]).  *total receives the normalized
 * byte count; if it exceeds out_capacity nothing is written and the call
 * returns SPM_RESOURCE_EXHAUSTED (allocate *total bytes and call again).
 * norm_to_orig is not produced.  One small read-back (the total). */
int spm_hip_normalize_batch_device(spm_hip_model *model, const uint8_t *d_in,
                                   const uint64_t *d_in_off, uint64_t n, uint8_t *d_out,
                                   uint64_t out_capacity, uint64_t *d_out_off, uint64_t *total,
                                   void *stream);

/* Pure stream version (no host synchronization): the normalized size is not
 * returned; if it exceeds out_capacity (3 * in_off[n] + 3 * n always
 * suffices) nothing is written and *d_status := SPM_RESOURCE_EXHAUSTED (see
 * spm_hip_encode_batch_async for the status-word contract).
 * d_norm_to_orig may be NULL (layout as in the _align variant below). */
int spm_hip_normalize_batch_device_async(spm_hip_model *model, const uint8_t *d_in,
                                         const uint64_t *d_in_off, uint64_t n, uint8_t *d_out,
                                         uint64_t out_capacity, uint64_t *d_out_off,
                                         uint32_t *d_norm_to_orig, uint32_t *d_status, void *stream);

/* Same, also producing norm_to_orig (Normalizer::Normalize's third output,
 * normalizer.cc:88-211): d_norm_to_orig receives, for sentence i, d_out_off
 * [i+1] - d_out_off[i] + 1 uint32 entries at d_norm_to_orig[d_out_off[i] + i]
 * (capacity out_capacity + n): the byte offset in the raw line of the
 * NormalizePrefix chunk each normalized byte came from, then the final
 * `consumed`.  Where the reference returns an empty vector (empty or
 * all-whitespace input) the single entry is the consumed byte count. */
int spm_hip_normalize_batch_device_align(spm_hip_model *model, const uint8_t *d_in,
                                         const uint64_t *d_in_off, uint64_t n, uint8_t *d_out,
                                         uint64_t out_capacity, uint64_t *d_out_off,
                                         uint32_t *d_norm_to_orig, uint64_t *total, void *stream);

/* One SentencePieceText::SentencePiece (sentencepiece.proto) as offsets:
 * piece = normalized[norm_begin, norm_end) of its sentence (empty for the
 * bos/eos pieces of the extra options: piece = IdToPiece(id)), surface =
 * raw line[begin, end). */
typedef struct spm_hip_piece {
  int32_t id;
  uint32_t begin, end;          /* byte offsets into the raw line */
  uint32_t norm_begin, norm_end;/* byte offsets into the normalized line */
} spm_hip_piece;

/* SentencePieceProcessor::Encode(input, SentencePieceText*) on the device
 * (sentencepiece_processor.cc:553-575): Normalize with norm_to_orig, model
 * Encode, PopulateSentencePieceText (:488-551: UNKNOWN runs merged, begin/end
 * through norm_to_orig) and ApplyExtraOptions (:945-979).  DEVICE pointers:
 * raw CSR in; normalized CSR out (capacity norm_capacity bytes, offsets
 * d_norm_off[n+1]); d_norm_to_orig (norm_capacity + n entries, layout as
 * above); pieces CSR out (capacity piece_capacity; d_piece_off[n+1]).
 * *total_norm / *total_pieces receive the sizes; if one exceeds its
 * capacity nothing further is written and SPM_RESOURCE_EXHAUSTED is
 * returned (norm_capacity + n * (bos/eos options) pieces always suffice). */
int spm_hip_encode_spt(spm_hip_model *model, const char *extra_options, const uint8_t *d_raw,
                       const uint64_t *d_raw_off, uint64_t n, uint8_t *d_norm, uint64_t norm_capacity,
                       uint64_t *d_norm_off, uint32_t *d_norm_to_orig, spm_hip_piece *d_pieces,
                       uint64_t piece_capacity, uint64_t *d_piece_off, uint64_t *total_norm,
                       uint64_t *total_pieces, void *stream);

/* Id epilogue of SentencePieceProcessor::Encode(ids) on the device:
 * PopulateSentencePieceText (sentencepiece_processor.cc:488-551 — runs of
 * UNKNOWN pieces merge into one id, :525-529) + ApplyExtraOptions (:945-979)
 * with the option string of SetEncodeExtraOptions ("bos:eos:reverse", parsed
 * as ParseExtraOptions :981-1010; NULL or "" = none).  DEVICE pointers:
 * d_ids / d_tok_offsets[n+1] as produced by spm_hip_encode_batch; output
 * d_out_ids (capacity out_capacity ids; tok_offsets[n] + n * (number of bos
 * and eos options) always suffices) and d_out_offsets[n+1].  *total (may be
 * NULL) receives the output id count; if it exceeds out_capacity nothing is
 * written and SPM_RESOURCE_EXHAUSTED is returned.  One small read-back. */
int spm_hip_finalize_ids(spm_hip_model *model, const char *extra_options, const int32_t *d_ids,
                         const uint64_t *d_tok_offsets, uint64_t n, int32_t *d_out_ids,
                         uint64_t out_capacity, uint64_t *d_out_offsets, uint64_t *total,
                         void *stream);

/* Pure stream version of spm_hip_finalize_ids (status-word contract of
 * spm_hip_encode_batch_async; the output count is in d_out_offsets[n]). */
int spm_hip_finalize_ids_async(spm_hip_model *model, const char *extra_options, const int32_t *d_ids,
                               const uint64_t *d_tok_offsets, uint64_t n, int32_t *d_out_ids,
                               uint64_t out_capacity, uint64_t *d_out_offsets, uint32_t *d_status,
                               void *stream);

/* Debug/testing knob: 1 = route every sentence through the exact general
 * kernel (reference-structured lattice), 0 = fast path with automatic
 * fallback (default). */
int spm_hip_model_set_force_general(spm_hip_model *model, int force);
/* 1 = record HIP events around each kernel launch (on the caller's stream)
 * and report their durations in spm_hip_encode_stats. */
int spm_hip_model_set_timing(spm_hip_model *model, int enable);
int spm_hip_model_last_stats(const spm_hip_model *model, spm_hip_encode_stats *stats);
/* Timing enabled: waits for `stream`, then returns the fast-kernel durations
 * (ms, HIP events on `stream`) of the encode calls made on it since the last
 * drain — at most the last 64 — oldest first, and resets the record. */
int spm_hip_model_drain_kernel_times(spm_hip_model *model, void *stream, float *ms, uint32_t capacity,
                                     uint32_t *count);
/* Debug/testing knob: the unigram fast kernel zeroes the EOS back-pointer of
 * sentence `sentence` (batch index; < 0 = off) after its forward pass, as a
 * corrupted scratch byte would.  The backtrace's bound check must turn that
 * into a general-kernel re-run of the sentence (exact output). */
int spm_hip_model_set_debug_corrupt_bp(spm_hip_model *model, int64_t sentence);
/* Tuning/testing knob: unigram models on the wide-char or char fast kernel
 * hand every sentence of at least `min_nb` normalized bytes to the
 * wave-cooperative kernel (one sentence per wavefront, coop_encode.hip);
 * 0 = never.  Default 128 (SPM_HIP_COOP_MIN_NB / SPM_HIP_COOP=0 at load).
 * Byte-kernel models ignore it. */
int spm_hip_model_set_coop_min_nb(spm_hip_model *model, uint32_t min_nb);
/* Tuning/testing knob: where the cooperative kernel's per-char scratch rows
 * live in a batch call.  mode 0 = automatic (rows by byte offset when the
 * call is smaller than the per-wave slabs, else one slab per wave), 1 =
 * always per-wave slabs, 2 = always by byte offset.  slab_chars = chars per
 * wave slab (0: the default 16384); a sentence of more chars goes to the
 * general kernel. */
int spm_hip_model_set_coop_slab(spm_hip_model *model, int mode, uint32_t slab_chars);
/* Releases the encode workspace (device scratch) kept for `stream` after
 * waiting for it.  A handle keeps at most 16 per-stream workspaces and
 * releases the least recently used idle one beyond that; each holds about
 * 13 bytes per normalized input byte of the largest batch seen on its
 * stream plus a 50 MB general-path pool. */
int spm_hip_model_release_stream(spm_hip_model *model, void *stream);

/* ---------------------------------------------------------------------------
 * Unigram trainer E-step (RunEStep, unigram_model_trainer.cc:237-287).
 * pieces: CSR of the TrainerModel piece list (value = list index), scores[V].
 * TrainerModel quirks reproduced: unk_id 0, max_score 0, all pieces NORMAL
 * (unigram_model_trainer.h:39-89).
 * mode: SPM_ESTEP_FAST  — per-sentence fp64 contributions reduced in fp64,
 *                         rounded to float once (not bit-equal to any thread
 *                         count of the reference; tolerance-checked);
 *       SPM_ESTEP_PARITY— emulates num_threads = T ordered float buckets, bit
 *                         exact against the reference at that T.
 * All pointers are DEVICE pointers; expected[V] float, obj float[1], ntok
 * int64[1] are written on `stream`.
 * ------------------------------------------------------------------------ */
enum spm_estep_mode { SPM_ESTEP_FAST = 0, SPM_ESTEP_PARITY = 1 };

typedef struct spm_hip_pieces spm_hip_pieces;

/* Builds the device trie for a piece list (host pointers). */
int spm_hip_pieces_create(const uint8_t *piece_bytes, const uint64_t *piece_offsets,
                          const float *scores, uint64_t num_pieces, spm_hip_pieces **out);
void spm_hip_pieces_free(spm_hip_pieces *pieces);
/* New scores for the same piece list (the next E-step when the M-step only
 * changed scores), keeping the trie and the work buffers.  No call on
 * `pieces` may be in flight on any stream.  num_pieces must equal the
 * create call's (else SPM_OUT_OF_RANGE).  Replaces rebuilding the
 * TrainerModel after each M-step (unigram_model_trainer.cc:97 SetSentencePieces,
 * called at :574) when the M-step kept every piece. */
int spm_hip_pieces_set_scores(spm_hip_pieces *pieces, const float *scores, uint64_t num_pieces);

int spm_hip_estep(spm_hip_pieces *pieces, const uint8_t *d_sent_bytes,
                  const uint64_t *d_sent_offsets, const int64_t *d_freq, uint64_t n,
                  int64_t all_sentence_freq, int mode, int num_threads,
                  float *d_expected, float *d_obj, int64_t *d_ntok, void *stream);

/* Split form for sharded (multi-GPU) E-steps.  The caller owns and zeroes the
 * accumulators and may all-reduce (sum) them across ranks between the two
 * calls (RCCL over xGMI):
 *   FAST  : acc = double[V], acc_obj = double[1], ntok_acc = int64[1]
 *   PARITY: acc = float[T*V] (bucket-major), acc_obj = float[T], ntok_acc = int64[T]
 * Sentence k of this call has global index index_base + k*index_stride; in
 * PARITY mode it belongs to bucket (global index mod T), and every sentence of
 * a bucket must be accumulated on one device, in ascending global order
 * (e.g. rank r of W with T == W passes the sentences r, r+W, ... with
 * index_base = r, index_stride = W).  Zero rows of other ranks' buckets make
 * a SUM all-reduce exact. */
int spm_hip_estep_accumulate(spm_hip_pieces *pieces, const uint8_t *d_sent_bytes,
                             const uint64_t *d_sent_offsets, const int64_t *d_freq, uint64_t n,
                             int64_t all_sentence_freq, int mode, int num_threads,
                             uint64_t index_base, uint64_t index_stride, void *d_acc,
                             void *d_acc_obj, int64_t *d_ntok_acc, void *stream);
int spm_hip_estep_finalize(spm_hip_pieces *pieces, int mode, int num_threads, const void *d_acc,
                           const void *d_acc_obj, const int64_t *d_ntok_acc, float *d_expected,
                           float *d_obj, int64_t *d_ntok, void *stream);
/* PARITY accumulation folds run on a library stream beside `stream`, and an
 * accumulate call normally makes `stream` wait for them before it returns.
 * With SPM_ESTEP_DEFER_FOLD or-ed into `mode`, the call returns without that
 * wait, so a caller feeding many calls (e.g. a corpus larger than its device
 * buffer) keeps the last fold of one call overlapped with the next call's
 * walks.  The accumulators are then complete on `stream` only after
 * spm_hip_estep_sync(pieces, stream) or spm_hip_estep_finalize (which syncs
 * first); read, reduce or free them only after one of the two. */
#define SPM_ESTEP_DEFER_FOLD 0x100
int spm_hip_estep_sync(spm_hip_pieces *pieces, void *stream);
const char *spm_hip_pieces_last_error(const spm_hip_pieces *pieces);
/* The E-step forward pass: 0 (default) the encode byte kernel's E-step mode
 * for accumulate calls of >= 2^20 sentences when the TrainerModel's pieces
 * are whole chars of < 16 bytes (else estep_forward_kernel); 1 that mode for
 * every call it applies to; 2 always estep_forward_kernel.  Results are
 * identical; this selects speed (and lets tests cover both passes). */
int spm_hip_pieces_set_forward(spm_hip_pieces *pieces, int mode);
/* PARITY record counts since the piece set was created: lattice-node records
 * written and records kept after the drop of provable no-ops (a record below
 * a quarter ulp of a lower bound of its float accumulator cannot change it;
 * estep_kernels.hip estep_threshold_kernel).  Diagnostics for the bench. */
int spm_hip_estep_record_stats(spm_hip_pieces *pieces, uint64_t *written, uint64_t *kept);
/* 1 = record HIP events around every accumulate chunk's forward pass and
 * backward pass on the caller's stream (bench roofline). */
int spm_hip_pieces_set_timing(spm_hip_pieces *pieces, int enable);
/* Timing enabled: waits for the recorded events and returns the summed
 * forward / backward pass durations (ms) and the chunk count since the last
 * call, releasing the events. */
int spm_hip_estep_kernel_times(spm_hip_pieces *pieces, double *forward_ms, double *backward_ms, uint64_t *chunks);

/* NBest(2) of PruneSentencePieces (unigram_model_trainer.cc:348-371, over
 * Lattice::NBest unigram_model.cc:339-477) for every piece of the list, on
 * the device, one piece per lane: the lattice of the piece's own string under
 * the TrainerModel, Viterbi, and the A* agenda with std::priority_queue's
 * exact heap order.  DEVICE pointers: the piece CSR (the list `pieces` was
 * created from, longest piece <= max_piece_bytes); d_keep[V]: 1 = always
 * keep, 0 = not, 2 = the search outgrew the device slab (caller re-runs that
 * piece on the host); d_alt at d_alt_off[i] (capacity: the piece's char
 * count) receives d_alt_n[i] ids of the second-best path when d_keep[i] == 1
 * (the reference's `alternatives`). */
int spm_hip_prune_nbest(spm_hip_pieces *pieces, const uint8_t *d_piece_bytes,
                        const uint64_t *d_piece_off, uint8_t *d_keep, int32_t *d_alt,
                        const uint64_t *d_alt_off, uint32_t *d_alt_n, uint32_t max_piece_bytes,
                        void *stream);

/* Shard plan of a W-rank E-step (spm_train --num_gpus; csrc/shard_plan.h):
 * rank `rank`'s segments as (index_base, index_stride, count) triples, the
 * arguments it passes to spm_hip_estep_accumulate.  Replaces the reference's
 * thread fan-out (unigram_model_trainer.cc:237-287, sentence i -> thread
 * i mod T) with bucket ownership per rank.  Writes at most `capacity`
 * triples into segs (3 * capacity uint64), the full count into *num_segments.
 * Host only (no device calls). */
int spm_hip_estep_shard_plan(uint64_t n, int mode, int num_threads, int world, int rank,
                             uint64_t *segs, uint64_t capacity, uint64_t *num_segments);

/* The rank that accumulates PARITY bucket `bucket` (0 <= bucket < num_threads)
 * under spm_hip_estep_shard_plan with `world` ranks — the rank spm_train's
 * cross-rank reduction gathers that float row from (RCCL send/recv or host
 * copy).  -1 on invalid arguments.  Host only. */
int spm_hip_estep_bucket_owner(int bucket, int num_threads, int world);

/* ---------------------------------------------------------------------------
 * Seed sentencepieces of the unigram trainer: MakeSeedSentencePieces
 * (unigram_model_trainer.cc:124-225, suffix array + internal nodes by esaxx,
 * esa.hxx:37-122), on the current HIP device.  HOST pointers in, results in
 * a host-side handle.
 *   sentences : CSR of the trainer's sentences after LoadSentences (normalized,
 *               rare chars replaced by U+2585), before the whitespace split
 *   chars / char_freq : the required chars with their freq-weighted counts
 *               (LoadSentences' chars_count restricted to required_chars_ —
 *               equal to the all_chars map of :131-139); every char of the
 *               sentences must be listed or be U+2585
 * Result (in seed order, ToLogProb applied): num_chars single chars sorted by
 * (count desc, UTF-8 asc), then substrings sorted by ((R-L)*D desc, suffix-
 * tree node index asc), up to seed_sentencepiece_size entries in total.
 * Limits: total chars + sentences < 2^32, sentences < 65535 chars,
 * max_sentencepiece_length <= 254.
 * ------------------------------------------------------------------------ */
typedef struct spm_hip_seed_options {
  int32_t max_sentencepiece_length;  /* TrainerSpec default 16 */
  int32_t split_by_unicode_script;   /* default 1 */
  int32_t split_by_number;           /* default 1 */
  int32_t split_by_whitespace;       /* default 1 */
  int32_t treat_whitespace_as_suffix;/* default 0 */
  int64_t seed_sentencepiece_size;   /* default 1000000 */
} spm_hip_seed_options;

typedef struct spm_hip_seeds spm_hip_seeds;

int spm_hip_seed_mine(const uint8_t *sent_bytes, const uint64_t *sent_offsets, uint64_t n,
                      const uint32_t *chars, const int64_t *char_freq, uint64_t num_chars,
                      const spm_hip_seed_options *opt, spm_hip_seeds **out);
/* Same with the sentences already in HBM (DEVICE pointers; chars/char_freq/
 * opt stay host pointers). */
int spm_hip_seed_mine_device(const uint8_t *d_sent_bytes, const uint64_t *d_sent_offsets, uint64_t n,
                             const uint32_t *chars, const int64_t *char_freq, uint64_t num_chars,
                             const spm_hip_seed_options *opt, spm_hip_seeds **out);
uint64_t spm_hip_seeds_size(const spm_hip_seeds *seeds);
const uint8_t *spm_hip_seeds_bytes(const spm_hip_seeds *seeds);     /* CSR values */
const uint64_t *spm_hip_seeds_offsets(const spm_hip_seeds *seeds);  /* size + 1 */
const float *spm_hip_seeds_scores(const spm_hip_seeds *seeds);      /* log-probs */
int spm_hip_seeds_stats(const spm_hip_seeds *seeds, uint64_t *num_chars, uint64_t *candidates,
                        float *device_ms);
/* Stage times of the substring pipeline (diagnostics): [0] upload + UTF-8
 * decode, [1] first radix sort (corpora split into parts: the split), [2]
 * the other sort passes (all rounds / parts), [3] capped
 * LCP + min pyramid + candidate nodes, [4] node sorts + gather + download
 * (device ms between stream events, host allocation gaps included), [5]
 * host wall ms inside hipMalloc, [6] prefix-doubling rounds. */
int spm_hip_seeds_stage_times(const spm_hip_seeds *seeds, float *ms, uint32_t capacity, uint32_t *count);
void spm_hip_seeds_free(spm_hip_seeds *seeds);
const char *spm_hip_seed_last_error(void);

/* ---------------------------------------------------------------------------
 * BPE trainer pair census (bpe::Trainer::Train, bpe_model_trainer.cc:200-230,
 * with the first UpdateActiveSymbols' ComputeFreq :87-113): the sentences
 * (DEVICE CSR + freq) decoded to code points, the unique chars and the unique
 * adjacent pairs in first-occurrence order (the reference's symbol creation
 * order), each pair's positions (EncodePos = sid << 32 | l << 16 | r, the
 * ones ComputeFreq keeps) and freq (sum of sentence freq over them).
 * Results live in a host-side handle.  Sentences of more than 65536 chars
 * return SPM_OUT_OF_RANGE (the reference CHECK-fails in EncodePos).
 * ------------------------------------------------------------------------ */
typedef struct spm_hip_bpe_census spm_hip_bpe_census;
int spm_hip_bpe_pair_census(const uint8_t *d_sent_bytes, const uint64_t *d_sent_offsets,
                            const int64_t *d_freq, uint64_t n, spm_hip_bpe_census **out,
                            void *stream);
void spm_hip_bpe_census_free(spm_hip_bpe_census *census);
const char *spm_hip_bpe_census_last_error(void);
/* Accessors (sizes via the *_size outputs). */
int spm_hip_bpe_census_view(const spm_hip_bpe_census *census, const uint32_t **char_codes,
                            const uint64_t **char_offsets, const uint32_t **unique_chars,
                            uint64_t *num_unique_chars, const uint64_t **pair_keys,
                            const uint64_t **pair_freq, const uint64_t **pair_pos_offsets,
                            const uint64_t **pair_positions, uint64_t *num_pairs, float *device_ms);

/* ---------------------------------------------------------------------------
 * BPE merge loop: the pair-frequency refresh of UpdateActiveSymbols
 * (bpe_model_trainer.cc:153-183 -> ComputeFreq :87-113, every bigram whose
 * freq was reset) on device-resident state.  create() uploads the sentences'
 * symbol ids (flat; sentence i = [sent_offsets[i], sent_offsets[i + 1]); -1 =
 * a char merged into its left neighbour), the sentence freqs and every
 * bigram's position set as (symbol id, EncodePos) entries sorted by (symbol,
 * position).  Each run() first applies the merge loop's changes since the
 * previous run -- symbol writes (flat index << 32 | uint32 value), positions
 * the host erased, positions inserted (sorted by (symbol, position); only
 * those still in the set) -- then recomputes the freq of every `todo`
 * symbol (triples: symbol id, left symbol id, right symbol id) exactly as
 * ComputeFreq does, erasing the positions it erases.  freq_out[k] is the
 * k-th todo symbol's freq; the erased positions come back as (symbol,
 * position) views valid until the next call; the caller removes them from its
 * own sets.  Host pointers throughout; one call = one upload, one
 * synchronization.
 * ------------------------------------------------------------------------ */
typedef struct spm_hip_bpe_refresh spm_hip_bpe_refresh;
int spm_hip_bpe_refresh_create(const int32_t *syms, const uint64_t *sent_offsets, const int64_t *sent_freq,
                               uint64_t num_sentences, const uint32_t *pos_sym, const uint64_t *pos_key,
                               uint64_t num_positions, void *stream, spm_hip_bpe_refresh **out);
int spm_hip_bpe_refresh_run(spm_hip_bpe_refresh *refresh, const uint64_t *sym_writes, uint64_t num_writes,
                            const uint32_t *ins_sym, const uint64_t *ins_key, uint64_t num_inserts,
                            const uint32_t *del_sym, const uint64_t *del_key, uint64_t num_erases,
                            const uint32_t *todo, uint64_t num_todo, uint64_t *freq_out,
                            const uint32_t **erased_sym, const uint64_t **erased_key, uint64_t *num_erased);
/* Entries held (alive or erased) and the device time of all runs so far. */
int spm_hip_bpe_refresh_stats(const spm_hip_bpe_refresh *refresh, uint64_t *num_entries, float *device_ms);
void spm_hip_bpe_refresh_free(spm_hip_bpe_refresh *refresh);

/* ---------------------------------------------------------------------------
 * Diagnostics (measurement only; not part of the reference surface).
 * Trie work of unigram Encode over a batch of normalized sentences (HOST
 * pointers), counted on host threads the way the reference's PopulateNodes
 * walks darts (unigram_model.cc:535-604, darts.h:469-512): one walk per char
 * start; every byte step is one dependent unit load (the mismatching probe
 * included), every matched leaf one value/score load.  units_below[k] counts
 * the unit loads that hit a unit index < (512 << k): how much of the walk an
 * LDS-resident top of the array of that size would serve.
 * ------------------------------------------------------------------------ */
typedef struct spm_hip_trie_stats {
  uint64_t char_starts;
  uint64_t unit_loads;
  uint64_t leaf_loads;
  uint64_t max_depth;
  uint64_t units_below[8];
  /* Wave-schedule model of the fast kernel (256-sentence blocks sorted by
   * length, 64-lane waves, byte positions walked in lockstep pairs): sum over
   * waves of the dependent load rounds, and the same if every lane walked its
   * own positions back to back (two chains per lane). */
  uint64_t lockstep_rounds;
  uint64_t decoupled_rounds;
  uint64_t waves;
} spm_hip_trie_stats;
int spm_hip_model_trie_stats(const spm_hip_model *model, const uint8_t *norm_bytes,
                             const uint64_t *offsets, uint64_t n, int num_threads,
                             spm_hip_trie_stats *out);

/* Raw lines -> the final ids of SentencePieceProcessor::Encode(line, &ids)
 * (sentencepiece_processor.cc:319-330: Normalizer::Normalize, normalizer.cc:
 * 88-211; ModelInterface::Encode, unigram_model.cc:705-720; the unknown-run
 * merge of PopulateSentencePieceText, :488-551) with no extra options, for
 * 1..16 lines of a unigram model in ONE device launch: raw image up and ids
 * down through pinned host memory, one completion word polled (the per-line
 * path of spm_encode_main.cc:189-191).  ids_cap entries in ids, n + 1 offsets
 * in out_off.  SPM_UNIMPLEMENTED: the fused path does not take this call (a
 * BPE model, more lines, a line of > 1024 bytes, a sentence whose lattice
 * needs the general kernel): run spm_hip_normalize_batch_device +
 * spm_hip_encode_batch + spm_hip_finalize_ids instead, nothing was written.
 * SPM_RESOURCE_EXHAUSTED: more ids than ids_cap (4 * raw bytes + 8 * n + 64
 * always suffices). */
int spm_hip_encode_raw_small_host(spm_hip_model *model, const uint8_t *raw, const uint64_t *raw_off,
                                  uint64_t n, int32_t *ids, uint64_t ids_cap, uint64_t *out_off);

/* Device memory this library holds in the calling process (every block it
 * allocates: models' workspaces, E-step piece sets, trainer corpus and
 * scratch): live bytes now and the high-water mark since the last reset.
 * No reference counterpart (the reference holds no device memory); bench.py
 * reports the peak per rank. */
int spm_hip_device_bytes(uint64_t *live, uint64_t *peak);
void spm_hip_device_peak_reset(void);

/* Human-readable message of the last error on this thread. */
const char *spm_hip_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SPM_HIP_H_ */
