/* C counterpart of the reference's examples/basic_tokenize.zig (same arguments, same
 * output format, :8-46), written against the C ABI (include/tkz.h). */
#include <stdio.h>
#include <string.h>

#include "tkz.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "Usage: %s <tokenizer.json> [text]\n", argv[0]);
        fprintf(stderr, "\nExample:\n");
        fprintf(stderr, "  %s path/to/tokenizer.json \"Hello, world!\"\n", argv[0]);
        return 0;
    }
    const char* path = argv[1];
    const char* text = argc > 2 ? argv[2] : "Hello, world!";
    fprintf(stderr, "Loading tokenizer from: %s\n", path);
    tkz_tokenizer* tk = NULL;
    int rc = tkz_create_from_file(path, &tk);
    if (rc) {
        fprintf(stderr, "error %d: %s\n", rc, tkz_last_error());
        return 1;
    }
    fprintf(stderr, "Tokenizing: \"%s\"\n\n", text);
    tkz_encoding enc;
    rc = tkz_encode(tk, (const uint8_t*)text, strlen(text), 1, &enc);
    if (rc) {
        fprintf(stderr, "error %d: %s\n", rc, tkz_last_error());
        tkz_destroy(tk);
        return 1;
    }
    fprintf(stderr, "Tokens (%zu):\n", enc.len);
    for (size_t i = 0; i < enc.len; ++i)
        fprintf(stderr, "  [%4zu] %6u = \"%.*s\"\n", i, enc.ids[i], (int)enc.token_lens[i], enc.tokens[i]);
    fprintf(stderr, "\nIDs: ");
    for (size_t i = 0; i < enc.len; ++i) fprintf(stderr, "%u ", enc.ids[i]);
    fprintf(stderr, "\n");
    tkz_encoding_free(&enc);
    tkz_destroy(tk);
    return 0;
}
