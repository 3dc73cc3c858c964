/*
 * tkz.h — C ABI of the MI355X-native batched tokenizer (drop-in for the encode hot
 * path of jrc2139/tokenizer-zig). Plain pointers and sizes only; no torch/HIP types.
 *
 * Each entry point names the reference interface it replaces (paths relative to the
 * reference repo, snapshot 2025-12-26). A Zig program binds this header with
 * @cImport; the Python mirror is tokenizer-zig_amd/tkz.
 *
 * Encode runs on the GPU (hand-written HIP kernels for gfx950). There is no CPU
 * fallback: on a machine without a usable MI355X every encode entry point returns
 * TKZ_ERR_DEVICE. Table construction, vocab queries and decode are host-side.
 */
#ifndef TKZ_H
#define TKZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes mirror the Zig error names (src/config.zig:18-30,
 * src/model/wordpiece.zig:150,212, std.fs errors of src/lib.zig:48-56). */
typedef enum tkz_status {
    TKZ_OK = 0,
    TKZ_ERR_INVALID_JSON = 1,            /* ConfigError.InvalidJson */
    TKZ_ERR_MISSING_MODEL = 2,           /* ConfigError.MissingModel */
    TKZ_ERR_UNSUPPORTED_MODEL_TYPE = 3,  /* ConfigError.UnsupportedModelType */
    TKZ_ERR_MISSING_VOCAB = 4,           /* ConfigError.MissingVocab */
    TKZ_ERR_INVALID_VOCAB_ENTRY = 5,     /* ConfigError.InvalidVocabEntry */
    TKZ_ERR_OUT_OF_MEMORY = 6,           /* error.OutOfMemory */
    TKZ_ERR_FILE_NOT_FOUND = 7,          /* error.FileNotFound (std.fs) */
    TKZ_ERR_FILE_TOO_BIG = 8,            /* error.FileTooBig (> 100 MiB, lib.zig:52) */
    TKZ_ERR_MISSING_UNK_TOKEN = 9,       /* error.MissingUnkToken (wordpiece.zig:150,212) */
    TKZ_ERR_INVALID_ARGUMENT = 10,       /* bad pointer / size / capacity */
    TKZ_ERR_DEVICE = 11                  /* no usable MI355X, or a HIP runtime error */
} tkz_status;

typedef struct tkz_tokenizer tkz_tokenizer;

/* Offset (src/types.zig:4-11). Offsets are byte offsets relative to the PRETOKEN the
 * token came from, exactly as Tokenizer.encode produces them (src/lib.zig:133-137). */
typedef struct tkz_offset {
    uint32_t start;
    uint32_t end;
} tkz_offset;

/* Encoding (src/encoding.zig:231-241). Arrays are library-allocated; free with
 * tkz_encoding_free. tokens[i]/token_lens[i] borrow the MODEL vocab's string of ids[i]
 * (Token.value: vocab_r.get(id), bpe.zig:255-262; added tokens never shadow it) and stay
 * valid until tkz_destroy. `words` is always NULL and `overflowing` always empty, as in
 * the reference (fromTokens). */
typedef struct tkz_encoding {
    size_t len;
    uint32_t* ids;
    uint32_t* type_ids;            /* all 0 */
    tkz_offset* offsets;
    uint32_t* special_token_mask;  /* all 0 */
    uint32_t* attention_mask;      /* all 1 */
    const char** tokens;
    uint32_t* token_lens;
} tkz_encoding;

/* CSR batch output: doc i's tokens are ids[row_ptr[i] .. row_ptr[i+1]). */
typedef struct tkz_batch {
    size_t n_docs;
    uint64_t n_tokens;
    uint64_t* row_ptr;     /* n_docs + 1 */
    uint32_t* ids;         /* n_tokens */
    tkz_offset* offsets;   /* n_tokens, pretoken-relative */
    /* set only when truncation or padding is enabled (else NULL: all 0 / 0 / 1) */
    uint32_t* type_ids;
    uint32_t* special_token_mask;
    uint32_t* attention_mask;
} tkz_batch;

/* Batched decode output: sequence i is bytes[offsets[i] .. offsets[i+1]). */
typedef struct tkz_text_batch {
    size_t n_docs;
    uint64_t n_bytes;
    uint64_t* offsets;     /* n_docs + 1 */
    char* bytes;           /* n_bytes (+ a terminating 0) */
} tkz_text_batch;

/* Parsed-config summary (what src/config.zig:59-117 installed). */
typedef struct tkz_info {
    int model;           /* 0 = WordPiece, 1 = BPE */
    int normalizer;      /* 0 = none, 1 = ASCII lowercase (BertNormalizer | Lowercase) */
    int pre_tokenizer;   /* 0 = none (whole text), 1 = Whitespace/WhitespaceSplit, 2 = BertPreTokenizer */
    int decoder;         /* 0 = none, 1 = WordPiece, 2 = ByteLevel, 3 = BPE */
    int has_post_processor;
    size_t model_vocab_size;
    size_t added_vocab_size;
    size_t n_merges;            /* accepted merges (BPE) */
    uint32_t unk_id;            /* 0xFFFFFFFF if none / not in vocab */
    uint64_t max_input_chars_per_word;  /* WordPiece */
    int compact_tables;         /* 1: 16-bit ids/ranks fast path */
    int merges_ordered;         /* 1: every merge ranks after the merges creating its parts
                                   (trained tables); 0: the segmented path never runs */
    int long_segments;          /* 1: long BPE pretokens take the segmented path
                                   (tkz_set_long_segments and merges_ordered) */
} tkz_info;

/* ---- construction (Tokenizer.fromJson / fromFile, src/lib.zig:48-85) ---------- */
int tkz_create_from_json(const char* json, size_t json_len, tkz_tokenizer** out);
int tkz_create_from_file(const char* path, tkz_tokenizer** out);
/* Creation options (SURVEY §8(b) tkz_opts): the device the tokenizer's tables and
 * workspaces live on (-1 = the device current at first GPU use), the BPE word memo
 * (tkz_set_word_memo), deferred-word dedup (tkz_set_dedup: -1 auto, 0 off, 1 on) and the
 * host-buffer pipeline chunk (tkz_set_host_pipeline, 0 = off). tkz_opts_default fills
 * the defaults that tkz_create_from_json uses. */
typedef struct tkz_opts {
    int device;
    int word_memo;
    int dedup;
    uint64_t host_chunk;
} tkz_opts;
void tkz_opts_default(tkz_opts* opts);
int tkz_create_from_json_opts(const char* json, size_t json_len, const tkz_opts* opts, tkz_tokenizer** out);
/* Tokenizer.deinit (src/lib.zig:87-106) */
void tkz_destroy(tkz_tokenizer* tk);
const char* tkz_last_error(void);          /* thread-local message of the last failure */
int tkz_get_info(const tkz_tokenizer* tk, tkz_info* out);

/* ---- encode (Tokenizer.encode, src/lib.zig:109-160) ---------------------------- */
/* One document -> Encoding. add_special_tokens has no effect, as in the reference
 * (the config post-processor is a no-op, src/config.zig:551-555). Runs the GPU path. */
int tkz_encode(tkz_tokenizer* tk, const uint8_t* text, size_t len, int add_special_tokens, tkz_encoding* out);
void tkz_encoding_free(tkz_encoding* enc);

/* Batched encode of host-resident docs: doc i is bytes[doc_off[i] .. doc_off[i+1]).
 * Equivalent to calling Tokenizer.encode on every doc. Output is library-allocated
 * host memory; free with tkz_batch_free. */
int tkz_encode_batch(tkz_tokenizer* tk, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                     tkz_batch* out);
void tkz_batch_free(tkz_batch* b);

/* tkz_encode_batch over several GPUs of this process (SURVEY §8(b) gpu_mask): bit i of
 * gpu_mask selects HIP device i. The docs are cut into one doc-aligned part per device
 * with about equal bytes; each part is encoded on its device from its own host thread, on
 * a replica of the tables uploaded to that device at first use (docs are independent:
 * Tokenizer.encode only reads the tables, lib.zig:109-160). The result is the same batch
 * tkz_encode_batch returns (row_ptr over all docs, parts concatenated). A bit naming a
 * device that does not exist fails with TKZ_ERR_INVALID_ARGUMENT; no device at all fails
 * with TKZ_ERR_DEVICE. Truncation / padding settings apply per encoding as usual. */
int tkz_encode_batch_gpus(tkz_tokenizer* tk, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                          uint32_t gpu_mask, tkz_batch* out);
/* Test hook for one-GPU machines: with n > 0, gpu_mask bit i maps to device i % (device
 * count), so several replicas share a device and the split / merge path runs. */
int tkz_set_virtual_devices(tkz_tokenizer* tk, int n);

/* Tokenizer.truncation / Tokenizer.padding (lib.zig:41-42, types.zig:39-59), applied by
 * tkz_encode / tkz_encode_batch after the (no-op) post-processor, as Tokenizer.encode steps
 * 6-7 (lib.zig:149-157): truncate each encoding to max_length, then pad it to `length`
 * (0 = no length: nothing to pad) with pad_id / pad_type_id / pad_token, on the right
 * (direction 0) or left (1). Pad positions: offsets (0,0), special 1, attention 0. Off by
 * default, as after fromJson. With max_length == length every row has exactly `length`
 * tokens: the CSR arrays are then a dense [n_docs, length] tensor. */
int tkz_set_truncation(tkz_tokenizer* tk, int enabled, size_t max_length, size_t stride);
int tkz_set_padding(tkz_tokenizer* tk, int enabled, size_t length, uint32_t pad_id, uint32_t pad_type_id,
                    const char* pad_token, size_t pad_token_len, int direction);
/* The same truncation/padding on a device-resident CSR batch (e.g. the output of
 * tkz_encode_batch_device); outputs sized by tkz_pad_capacity, asynchronous on `stream`. */
uint64_t tkz_pad_capacity(const tkz_tokenizer* tk, size_t n_docs, uint64_t n_tokens);
size_t tkz_pad_workspace_size(size_t n_docs);
int tkz_pad_batch_device(tkz_tokenizer* tk, const uint64_t* d_row_ptr, const uint32_t* d_ids,
                         const tkz_offset* d_offsets, size_t n_docs, uint64_t* d_row_ptr2, uint32_t* d_ids2,
                         tkz_offset* d_offsets2, uint32_t* d_type_ids, uint32_t* d_special_mask,
                         uint32_t* d_attention_mask, void* d_workspace, size_t workspace_bytes, void* stream);

/* Batched encode of DEVICE-resident docs on `stream` (a hipStream_t, NULL = the
 * tokenizer's own stream). No allocation.
 *   d_bytes:   total_bytes bytes, buffer readable up to a multiple of 16 bytes
 *   d_doc_off: n_docs + 1 offsets (uint64) into d_bytes
 *   d_row_ptr: n_docs + 1 (written); d_row_ptr[n_docs] = total tokens
 *   d_ids / d_offsets: capacity >= total_bytes entries (tokens never exceed bytes)
 *   d_workspace: workspace_bytes >= tkz_device_workspace_min(). With
 *              >= tkz_device_workspace_size(total_bytes, n_docs) bytes (about 27 B per input
 *              byte + 16 MB) the batch runs in one pass, asynchronously (no host sync).
 *              With less, it runs in doc-aligned sub-batches of the largest size the
 *              workspace supports (tkz_device_workspace_size_sub(B) holds sub-batches of B
 *              bytes); the outputs are the same. The host then waits once per 4096
 *              sub-batches for the cut points (read from d_doc_off on the device). A
 *              single document larger than a sub-batch fails with TKZ_ERR_INVALID_ARGUMENT.
 *              One pass is limited to 2^36 bytes (64 GiB); larger batches are sub-batched.
 *   d_status:  one uint32 set to a tkz_status != 0 on a device-detected error
 *              (MissingUnkToken); zero it before the call. */
size_t tkz_device_workspace_size(const tkz_tokenizer* tk, uint64_t total_bytes, size_t n_docs);
size_t tkz_device_workspace_size_sub(const tkz_tokenizer* tk, uint64_t sub_batch_bytes);
size_t tkz_device_workspace_min(const tkz_tokenizer* tk);
int tkz_encode_batch_device(tkz_tokenizer* tk, const uint8_t* d_bytes, const uint64_t* d_doc_off, size_t n_docs,
                            uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, tkz_offset* d_offsets,
                            void* d_workspace, size_t workspace_bytes, uint32_t* d_status, void* stream);

/* Statistics of the last encode that used workspace d_workspace (NULL = the tokenizer's
 * own workspace, i.e. the last tkz_encode_batch): pretokens, pretokens resolved by the
 * BPE word memo / WordPiece whole-word probe, memo-missing BPE words deferred to the
 * long-word kernel (and how many of them the model ran on after dedup), the number
 * of passes (sub-batches), and the words of > 64 bytes (one wavefront each). Waits for
 * all work of the tokenizer's device first (hipDeviceSynchronize on that device, whichever
 * device the calling thread has current), so no stream sync is needed.
 * tkz_device_batch_stats_stream waits for `stream` only (the stream the encode ran on;
 * NULL = the tokenizer's own stream): no barrier across the device's other streams. */
typedef struct {
    uint64_t pretokens;
    uint64_t memo_hits;
    uint64_t deferred;
    uint64_t deferred_model;
    uint64_t sub_batches;
    uint64_t long_words;   /* BPE words of > 64 bytes run by the wave-cooperative kernels */
    uint64_t long_segmented; /* ... of which the segmented path encoded (tkz_set_long_segments) */
    uint64_t long_fallback_bytes; /* bytes of the long words the one-wave-per-word kernel ran on (those
                                     the segmented path left, or all of them with it off) */
    uint64_t seg_bound_errors;    /* debug builds (-DTKZ_SEG_BOUNDS=1): bounds the segmented path's
                                     kernels found exceeded (bit per check); always 0 otherwise */
} tkz_batch_stats;
int tkz_device_batch_stats(const tkz_tokenizer* tk, const void* d_workspace, tkz_batch_stats* out);
int tkz_device_batch_stats_stream(const tkz_tokenizer* tk, const void* d_workspace, void* stream,
                                  tkz_batch_stats* out);

/* ---- decode & vocab (src/lib.zig:163-223) -------------------------------------- */
/* Tokenizer.decode (lib.zig:163-189) + config decoders (config.zig:488-530). Host-side.
 * *out is NUL-terminated, library-allocated; free with tkz_string_free. */
int tkz_decode(const tkz_tokenizer* tk, const uint32_t* ids, size_t n, int skip_special_tokens, char** out,
               size_t* out_len);
void tkz_string_free(char* s);
/* Batched Tokenizer.decode on the GPU: sequence i is ids[row_ptr[i] .. row_ptr[i+1]), each
 * decoded exactly as tkz_decode / lib.zig:163-189 would (config decoder applied per
 * sequence). Host buffers in, library-allocated output; free with tkz_text_batch_free. */
int tkz_decode_batch(tkz_tokenizer* tk, const uint64_t* row_ptr, const uint32_t* ids, size_t n_docs,
                     int skip_special_tokens, tkz_text_batch* out);
void tkz_text_batch_free(tkz_text_batch* b);
/* Device-resident batched decode on `stream` (NULL = the tokenizer's stream), asynchronous:
 *   d_row_ptr n_docs + 1, d_ids n_tokens (device); d_out >= tkz_decode_bound(n_tokens)
 *   bytes; d_out_off n_docs + 1 (written; d_out_off[n_docs] = total bytes);
 *   d_workspace >= tkz_decode_workspace_size(n_docs, n_tokens) bytes. */
uint64_t tkz_decode_bound(const tkz_tokenizer* tk, uint64_t n_tokens);
size_t tkz_decode_workspace_size(const tkz_tokenizer* tk, size_t n_docs, uint64_t n_tokens);
int tkz_decode_batch_device(tkz_tokenizer* tk, const uint64_t* d_row_ptr, const uint32_t* d_ids, size_t n_docs,
                            uint64_t n_tokens, int skip_special_tokens, uint8_t* d_out, uint64_t out_capacity,
                            uint64_t* d_out_off, void* d_workspace, size_t workspace_bytes, void* stream);
/* Tokenizer.getVocabSize (lib.zig:203-205): model vocab + added tokens. */
size_t tkz_get_vocab_size(const tkz_tokenizer* tk);
/* Tokenizer.tokenToId (lib.zig:208-214): returns 1 and sets *id if found, else 0. */
int tkz_token_to_id(const tkz_tokenizer* tk, const char* token, size_t len, uint32_t* id);
/* Tokenizer.idToToken (lib.zig:217-223): NULL if unknown. Borrowed; valid until destroy. */
const char* tkz_id_to_token(const tkz_tokenizer* tk, uint32_t id, size_t* len);
/* Tokenizer.addSpecialTokens (lib.zig:192-200): returns the number newly added. Each token
 * gets the next free added-vocab id (AddedToken.id = null, vocab.zig:44). */
size_t tkz_add_special_tokens(tkz_tokenizer* tk, const char* const* tokens, const size_t* lens, size_t n);
/* The same with AddedToken.id per token (ids[i] == TKZ_NO_ID: null); ids may be NULL. */
#define TKZ_NO_ID 0xFFFFFFFFu
size_t tkz_add_special_tokens_ids(tkz_tokenizer* tk, const char* const* tokens, const size_t* lens,
                                  const uint32_t* ids, size_t n);

/* ---- FastTokenizer API (src/lib.zig:236-454, SpanEncoding src/encoding.zig:16-224) -- */
/* FastTokenizerOptions (lib.zig:237-242); C default {8192, 512}. */
typedef struct tkz_fast_options {
    uint32_t max_sequence_length; /* pretoken cap = max_sequence_length / 4 per doc (arena.zig:192) */
    uint32_t max_tokens;          /* SpanEncoding capacity (arena.zig:179) */
} tkz_fast_options;

/* A batch of SpanEncodings as dense rows: doc d is ids[d*capacity .. d*capacity+len[d]).
 * Entries past len[d] are 0 (ids, offsets) and attention_mask is 1 / 0; type_ids are 0
 * (SpanToken.type_id default, token.zig:28). Library-allocated; free with tkz_span_batch_free. */
typedef struct tkz_span_batch {
    size_t n_docs;
    uint32_t capacity;         /* max_tokens */
    uint32_t* len;             /* [n_docs] */
    uint32_t* ids;             /* [n_docs * capacity] */
    tkz_offset* offsets;       /* [n_docs * capacity], pretoken-relative like the reference */
    uint32_t* attention_mask;  /* [n_docs * capacity] */
} tkz_span_batch;

/* FastTokenizer.encode (lib.zig:352-413) over a batch of docs. Same caps as the reference:
 * only the first max_sequence_length/4 pretokens of a doc are tokenized and at most
 * max_tokens tokens are kept (SpanEncoding.tryAppend). The tokens themselves are those of
 * Tokenizer.encode (the exact slow path; intentional difference: BPE.tokenizeFast's heap
 * order can give other ids, bpe.zig:285-430), and a WordPiece word that needs a missing
 * UNK yields no token, as WordPiece.tokenizeFast does (wordpiece.zig:241,297). */
int tkz_fast_encode_batch(tkz_tokenizer* tk, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                          const tkz_fast_options* opts, tkz_span_batch* out);
void tkz_span_batch_free(tkz_span_batch* b);
/* Device-resident variant on `stream` (NULL = the tokenizer's stream), asynchronous.
 *   max_doc_bytes: the longest doc if known (0 = unknown); when it is <= the pretoken cap the
 *   input is read in place, otherwise a clipped copy is made in the workspace.
 *   d_len [n_docs]; d_ids, d_offsets, d_attention_mask (may be NULL) [n_docs * max_tokens];
 *   d_workspace >= tkz_fast_workspace_size(...) bytes; d_status as tkz_encode_batch_device. */
size_t tkz_fast_workspace_size(const tkz_tokenizer* tk, uint64_t total_bytes, size_t n_docs);
int tkz_fast_encode_batch_device(tkz_tokenizer* tk, const uint8_t* d_bytes, const uint64_t* d_doc_off,
                                 size_t n_docs, uint64_t total_bytes, uint64_t max_doc_bytes,
                                 const tkz_fast_options* opts, uint32_t* d_len, uint32_t* d_ids,
                                 tkz_offset* d_offsets, uint32_t* d_attention_mask, void* d_workspace,
                                 size_t workspace_bytes, uint32_t* d_status, void* stream);

/* BPE word memo (default on): the BPE result of every vocab key of <= 16 bytes is
 * computed once by the GPU encode path when the tables are uploaded; a pretoken equal
 * to such a key then reuses it (bit-identical by construction). 0 disables it. */
int tkz_set_word_memo(tkz_tokenizer* tk, int on);

/* The memos' size on the device: keys held by the word memo (vocab keys and their
 * capitalised / punctuated variants whose tokens fit a slot) and the bytes of every memo
 * table -- the word memo's two tables, the segment memo (table + pool) and the hot-pair
 * bitmap; 0 / 0 when the memo is off or not built yet (it is built at the first GPU use). */
int tkz_get_memo_info(const tkz_tokenizer* tk, uint64_t* entries, uint64_t* table_bytes);
/* The same, table by table, with the hot-pair bitmap's keys and build time. */
typedef struct tkz_memo_info {
    uint64_t word_entries, word_bytes;  /* BPE word memo */
    uint64_t seg_entries, seg_bytes;    /* segment memo of the segmented path (table + pool) */
    uint64_t hot_keys, hot_bitmap_bytes; /* hot-pair bitmap: hot_keys^2 bits */
    double hot_build_ms;                /* its build at table load (k_seg_hot_build) */
} tkz_memo_info;
int tkz_get_memo_info_ext(const tkz_tokenizer* tk, tkz_memo_info* out);
/* Keys of the segmented path's hot-pair bitmap (a precomputed boundary check for every
 * ordered pair of the max_keys most frequent memo keys: max_keys^2 / 8 bytes of device
 * memory). -1 = default: the TKZ_HOT_K environment variable, else 65,536 (512 MB, ~0.1 s
 * to build); 0 = none. Always capped at 1/64 of the device's free memory when built.
 * Applies at the tables' first GPU use, or rebuilds the bitmap at once when they are
 * built. Results are the same with any value. */
int tkz_set_hot_pairs(tkz_tokenizer* tk, int64_t max_keys);

/* Deduplication of the BPE words the word memo does not resolve (GPU batches): each
 * distinct word of <= 32 bytes runs the model once per batch and its repeats copy the
 * result (bit-identical by construction). mode: -1 auto (default; on when the vocab has
 * >= 256 multi-byte characters), 0 off, 1 on. */
int tkz_set_dedup(tkz_tokenizer* tk, int mode);

/* tkz_encode_batch without truncation / padding overlaps its PCIe copies: batches of at
 * least 2 x chunk_bytes input bytes go in doc-aligned chunks, the input copy and encode of
 * one chunk running while the CSR output of the previous one is copied back. The host
 * arrays are sized from the previous batch's tokens per byte, so the first batch of a
 * tokenizer runs unchunked. Results are identical. 0 disables; default 32 MiB; sizes
 * below 1 MiB are raised to 1 MiB (each chunk is a full launch sequence). */
int tkz_set_host_pipeline(tkz_tokenizer* tk, size_t chunk_bytes);

/* ---- device / table introspection (tests, tools) ------------------------------- */
int tkz_device_available(void);  /* 1 if a GPU is usable from this process */
/* Long BPE pretokens (> 64 B: the whole text under a ByteLevel / Metaspace / unknown
 * pre_tokenizer, config.zig:387-402) are cut into segments encoded independently: at the
 * ASCII chars BPE.tokenize skips (no id, no unk: bpe.zig:192-208), around ASCII chars whose
 * symbol (own id or the unk id) is in no merge (never crossed), and before ASCII whitespace
 * with a mergeable id; every other cut is checked exactly against the merge order and the
 * segments a merge crosses are re-encoded together. Compact tables and wide ones with ids
 * < 2^20 - 1 (on by default; the results are the same either way; on != 0 turns it on).
 * The boundary check assumes every merge ranks after the merges that create its parts
 * (true of any trained merge list); a merge table where that fails never takes the path,
 * whatever `on` says (tkz_info.merges_ordered / long_segments report it). */
int tkz_set_long_segments(tkz_tokenizer* tk, int on);
/* Selects the HIP device used by tokenizers first used on this thread afterwards
 * (one process per GPU: pass LOCAL_RANK). */
int tkz_set_device(int device);
/* Looks (a,b) up in the GPU merge table image (host copy): 1 + rank/new_id if present. */
int tkz_debug_merge_lookup(const tkz_tokenizer* tk, uint32_t a, uint32_t b, uint32_t* rank, uint32_t* new_id);
/* Looks a vocab key up in the GPU WordPiece/char table image (host copy). */
int tkz_debug_vocab_lookup(const tkz_tokenizer* tk, const char* key, size_t len, uint32_t* id);
/* Offset in the device workspace of the kernel debug counters (profiling builds). */
size_t tkz_debug_counters_offset(uint64_t total_bytes, size_t n_docs);

/* ---- plumbing for benches and tests (device memory, sync, kernel timers) -------- */
void* tkz_dev_alloc(size_t n);
void tkz_dev_free(void* p);
int tkz_memcpy_htod(void* dst, const void* src, size_t n);
int tkz_memcpy_dtoh(void* dst, const void* src, size_t n);
int tkz_memset_dev(void* dst, int value, size_t n);
/* Free and total bytes of the current device (hipMemGetInfo): sizes a workspace cap. */
int tkz_dev_mem_info(size_t* free_bytes, size_t* total_bytes);
int tkz_synchronize(tkz_tokenizer* tk);   /* waits for the tokenizer's stream */
/* A non-blocking HIP stream on the current device (hipStream_t as void*), for batches in
 * flight on several streams (tkz_encode_batch_device); null on failure. */
void* tkz_stream_create(void);
void tkz_stream_destroy(void* stream);
int tkz_device_synchronize(void);        /* waits for all work on the current device */
/* Records HIP events around each kernel group of every encode call on its stream. */
int tkz_profile_enable(tkz_tokenizer* tk, int on);
/* ms[0] = k_encode, ms[1] = k_bpe_deferred (long BPE words), ms[2] = count + scan,
 * ms[3] = compaction, summed over the calls recorded since the last reset (call after
 * tkz_synchronize). */
int tkz_profile_read(tkz_tokenizer* tk, double* ms, uint64_t* n_calls, int reset);
/* Timeline of the pipelined host-buffer path (tkz_encode_batch), recorded while profiling
 * is on, summed over calls: out[0] calls, [1] chunks, [2] input bytes, [3] output bytes,
 * then ms: [4] wall time of the calls, [5] output allocation, [6] host waits for chunk
 * counts, [7] row_ptr fix-up, [8] input copies (sum over chunks), [9] encodes, [10] output
 * copies, [11] / [12] / [13] first-to-last spans of the input copies / encodes / output
 * copies, [14] first chunk in + encoded, [15] last chunk's output copy. n <= 16 fields. */
int tkz_host_profile_read(tkz_tokenizer* tk, double* out, size_t n, int reset);
/* Page-locked host memory (hipHostMalloc): input text staged here reaches the device at
 * the full PCIe rate in tkz_encode_batch (pageable input goes through the runtime's
 * bounce buffers). Optional: any host buffer is accepted. */
void* tkz_host_alloc(size_t n);
void tkz_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* TKZ_H */
