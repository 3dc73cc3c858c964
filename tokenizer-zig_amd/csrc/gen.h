/* libtkzgen.so: device-side bench / test utilities (gen.hip). Not the encode path and
 * not part of the product ABI (include/tkz.h); used by bench.py and the GPU tests. */
#ifndef TKZ_GEN_H
#define TKZ_GEN_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct tkz_gen tkz_gen;
/* Uploads the generator tables of one config (tkz_synth_tables in libtkzsynth.so):
 * p = {kind, fixed_len, zmin, n_words, n_cps, n_len}. Returns 0 on success. */
int tkz_gen_create(const int64_t* p, const uint32_t* wcp, const uint32_t* woff, const double* wcdf,
                   const double* lcdf, tkz_gen** out);
void tkz_gen_destroy(tkz_gen* g);
/* doc_off[0..n_docs] of docs [first_doc, first_doc + n_docs) on the device; *total = the
 * byte count (synchronous). */
int tkz_gen_offsets(tkz_gen* g, uint64_t seed, uint64_t first_doc, uint64_t n_docs, uint64_t* d_doc_off,
                    uint64_t* total, void* stream);
/* The docs' bytes at d_out[d_doc_off[i] ..], byte-identical to tkz_synth_docs (synchronous). */
int tkz_gen_bytes(tkz_gen* g, uint64_t seed, uint64_t first_doc, uint64_t n_docs, const uint64_t* d_doc_off,
                  uint8_t* d_out, void* stream);
/* Rolling hashes (tests/shard_hash.py) of a device CSR batch: out = {row_ptr (n_docs + 1
 * values), ids (u32 as u64), offsets (start | end << 32)}. Synchronous. */
int tkz_csr_hash_device(const uint64_t* d_row_ptr, uint64_t n_docs, const uint32_t* d_ids, const uint64_t* d_offsets,
                        uint64_t n_tokens, uint64_t out[3], void* stream);
#ifdef __cplusplus
}
#endif
#endif
