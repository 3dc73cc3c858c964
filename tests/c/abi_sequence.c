/* The call sequence of integration/zig/gpu.zig (the reference's Tokenizer API,
 * /root/reference/src/lib.zig:48-223) made through the C ABI (include/tkz.h):
 *   fromJson, fromFile, getVocabSize, tokenToId, idToToken, decode, addSpecialTokens,
 *   [gpu: encode, encodeBatch, decodeBatch], the error paths, deinit.
 * Prints one JSON object; tests/test_abi_sequence.py checks it against the reference's
 * golden vectors and the oracle. Strings are printed as byte arrays.
 *
 * usage: abi_sequence <tokenizer.json> host|gpu <text> <tok1,tok2,...> <id1,id2,...> */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tkz.h"

static void put_bytes(const char* key, const char* p, size_t n) {
    printf("\"%s\": [", key);
    for (size_t i = 0; i < n; ++i) printf("%s%u", i ? ", " : "", (unsigned)(unsigned char)p[i]);
    printf("], ");
}

static void put_u32s(const char* key, const uint32_t* p, size_t n) {
    printf("\"%s\": [", key);
    for (size_t i = 0; i < n; ++i) printf("%s%u", i ? ", " : "", p[i]);
    printf("], ");
}

static char* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)sz + 1);
    *n = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    return buf;
}

/* comma-separated list -> array of strings (in place) */
static size_t split(char* s, char** out, size_t cap) {
    size_t n = 0;
    if (!*s) return 0;
    for (char* p = s; n < cap;) {
        out[n++] = p;
        char* c = strchr(p, ',');
        if (!c) break;
        *c = 0;
        p = c + 1;
    }
    return n;
}

static void put_decode(const char* key, tkz_tokenizer* tk, const uint32_t* ids, size_t n, int skip) {
    char* s = NULL;
    size_t len = 0;
    int rc = tkz_decode(tk, ids, n, skip, &s, &len);
    if (rc) { printf("\"%s\": {\"error\": %d}, ", key, rc); return; }
    put_bytes(key, s, len);
    tkz_string_free(s);
}

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s <tokenizer.json> host|gpu <text> <tokens> <ids>\n", argv[0]);
        return 2;
    }
    const int gpu = strcmp(argv[2], "gpu") == 0;
    const char* text = argv[3];
    char* toks[64];
    char* idstr[64];
    const size_t nt = split(argv[4], toks, 64), ni = split(argv[5], idstr, 64);
    uint32_t ids[64];
    for (size_t i = 0; i < ni; ++i) ids[i] = (uint32_t)strtoul(idstr[i], NULL, 10);
    size_t jn = 0;
    char* js = read_file(argv[1], &jn);
    if (!js) { fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }

    printf("{");
    /* Tokenizer.fromJson / fromFile (lib.zig:48-85) */
    tkz_tokenizer* tk = NULL;
    int rc = tkz_create_from_json(js, jn, &tk);
    printf("\"from_json\": %d, ", rc);
    if (rc) { printf("\"msg\": \"%s\"}\n", tkz_last_error()); return 1; }
    tkz_tokenizer* tf = NULL;
    rc = tkz_create_from_file(argv[1], &tf);
    printf("\"from_file\": %d, \"from_file_vocab_size\": %zu, ", rc, rc ? 0 : tkz_get_vocab_size(tf));
    if (!rc) tkz_destroy(tf);

    /* getVocabSize / tokenToId / idToToken (lib.zig:203-223) */
    printf("\"vocab_size\": %zu, ", tkz_get_vocab_size(tk));
    printf("\"token_to_id\": [");
    for (size_t i = 0; i < nt; ++i) {
        uint32_t id = 0;
        int found = tkz_token_to_id(tk, toks[i], strlen(toks[i]), &id);
        if (found) printf("%s%u", i ? ", " : "", id);
        else printf("%snull", i ? ", " : "");
    }
    printf("], \"id_to_token\": [");
    for (size_t i = 0; i < ni; ++i) {
        size_t len = 0;
        const char* s = tkz_id_to_token(tk, ids[i], &len);
        printf("%s", i ? ", " : "");
        if (!s) { printf("null"); continue; }
        printf("[");
        for (size_t k = 0; k < len; ++k) printf("%s%u", k ? ", " : "", (unsigned)(unsigned char)s[k]);
        printf("]");
    }
    printf("], ");

    /* decode (lib.zig:163-189) */
    put_decode("decode", tk, ids, ni, 0);
    put_decode("decode_skip", tk, ids, ni, 1);

    /* addSpecialTokens (lib.zig:192-200): a new token, one with an explicit id, a repeat */
    const char* sp[3] = {"<x1>", "<x2>", "<x1>"};
    const size_t sl[3] = {4, 4, 4};
    const uint32_t sid[3] = {TKZ_NO_ID, 500, TKZ_NO_ID};
    printf("\"added\": %zu, ", tkz_add_special_tokens_ids(tk, sp, sl, sid, 3));
    uint32_t x2 = 0;
    printf("\"x2_id\": %d, ", tkz_token_to_id(tk, "<x2>", 4, &x2) ? (int)x2 : -1);
    printf("\"vocab_size_after\": %zu, ", tkz_get_vocab_size(tk));
    uint32_t with_x2[65];
    memcpy(with_x2, ids, ni * 4);
    with_x2[ni] = 500;
    put_decode("decode_x2", tk, with_x2, ni + 1, 0);
    put_decode("decode_x2_skip", tk, with_x2, ni + 1, 1);

    if (gpu) {
        /* encode (lib.zig:109-160) */
        tkz_encoding e;
        rc = tkz_encode(tk, (const uint8_t*)text, strlen(text), 1, &e);
        printf("\"encode\": %d, ", rc);
        if (!rc) {
            put_u32s("ids", e.ids, e.len);
            put_u32s("type_ids", e.type_ids, e.len);
            put_u32s("special_token_mask", e.special_token_mask, e.len);
            put_u32s("attention_mask", e.attention_mask, e.len);
            printf("\"offsets\": [");
            for (size_t i = 0; i < e.len; ++i) printf("%s[%u, %u]", i ? ", " : "", e.offsets[i].start, e.offsets[i].end);
            printf("], \"tokens\": [");
            for (size_t i = 0; i < e.len; ++i) {
                printf("%s[", i ? ", " : "");
                for (uint32_t k = 0; k < e.token_lens[i]; ++k)
                    printf("%s%u", k ? ", " : "", (unsigned)(unsigned char)e.tokens[i][k]);
                printf("]");
            }
            printf("], ");
            tkz_encoding_free(&e);
        }
        /* batch: [text, text, ""] and its decode */
        const size_t L = strlen(text);
        uint8_t* buf = (uint8_t*)calloc(2 * L + 16, 1);
        memcpy(buf, text, L);
        memcpy(buf + L, text, L);
        uint64_t off[4] = {0, L, 2 * L, 2 * L};
        tkz_batch b;
        rc = tkz_encode_batch(tk, buf, off, 3, &b);
        printf("\"encode_batch\": %d, ", rc);
        if (!rc) {
            printf("\"batch_row_ptr\": [%llu, %llu, %llu, %llu], ", (unsigned long long)b.row_ptr[0],
                   (unsigned long long)b.row_ptr[1], (unsigned long long)b.row_ptr[2],
                   (unsigned long long)b.row_ptr[3]);
            put_u32s("batch_ids", b.ids, b.n_tokens);
            tkz_text_batch tb;
            rc = tkz_decode_batch(tk, b.row_ptr, b.ids, 3, 0, &tb);
            printf("\"decode_batch\": %d, ", rc);
            if (!rc) {
                put_bytes("decode_batch_row0", tb.bytes + tb.offsets[0], tb.offsets[1] - tb.offsets[0]);
                printf("\"decode_batch_row2_len\": %llu, ", (unsigned long long)(tb.offsets[3] - tb.offsets[2]));
                tkz_text_batch_free(&tb);
            }
            tkz_batch_free(&b);
        }
        free(buf);
    } else {
        /* without a GPU, encode fails loudly (no CPU fallback) */
        tkz_encoding e;
        rc = tkz_encode(tk, (const uint8_t*)text, strlen(text), 1, &e);
        printf("\"encode\": %d, ", rc);
        if (!rc) tkz_encoding_free(&e);
    }

    /* error paths (config.zig:18-30, lib.zig:48-56) */
    tkz_tokenizer* bad = NULL;
    const char* e1 = "{";
    const char* e2 = "{\"model\":{\"type\":\"BPE\",\"vocab\":{\"a\":0,\"a\":1}}}";
    const char* e3 = "{}";
    const char* e4 = "{\"model\":{\"type\":\"Unigram\",\"vocab\":{}}}";
    printf("\"err_invalid_json\": %d, ", tkz_create_from_json(e1, strlen(e1), &bad));
    printf("\"err_duplicate_key\": %d, ", tkz_create_from_json(e2, strlen(e2), &bad));
    printf("\"err_missing_model\": %d, ", tkz_create_from_json(e3, strlen(e3), &bad));
    printf("\"err_unsupported\": %d, ", tkz_create_from_json(e4, strlen(e4), &bad));
    printf("\"err_file\": %d, ", tkz_create_from_file("/nonexistent/tokenizer.json", &bad));

    /* deinit (lib.zig:87-106) */
    tkz_destroy(tk);
    free(js);
    printf("\"done\": true}\n");
    return 0;
}
