//! GpuTokenizer: the reference's `Tokenizer` API (src/lib.zig:32-224 of
//! jrc2139/tokenizer-zig) over the C ABI of include/tkz.h, for a maintainer to drop into
//! the reference tree as src/gpu.zig (build wiring: INTEGRATION.md). Every method keeps
//! the reference's name, arguments, ownership and error names; encode runs the MI355X
//! kernels. Not compiled in this repository (no Zig toolchain in the build image):
//! tests/c/abi_sequence.c makes the same C calls in the same order and is run by
//! tests/test_abi_sequence.py (host calls on CPU, encode / decode batches on the GPU).
const std = @import("std");
const c = @cImport(@cInclude("tkz.h"));
const Encoding = @import("encoding.zig").Encoding;
const Offset = @import("types.zig").Offset;
const AddedToken = @import("types.zig").AddedToken;
const TruncationParams = @import("types.zig").TruncationParams;
const PaddingParams = @import("types.zig").PaddingParams;

/// The reference's error names (config.zig:18-30, wordpiece.zig:150,212, std.fs), plus
/// DeviceError (no usable MI355X / HIP failure) and InvalidArgument.
pub const Error = error{
    InvalidJson,
    MissingModel,
    UnsupportedModelType,
    MissingVocab,
    InvalidVocabEntry,
    OutOfMemory,
    FileNotFound,
    FileTooBig,
    MissingUnkToken,
    InvalidArgument,
    DeviceError,
};

fn mapError(rc: c_int) Error {
    return switch (rc) {
        c.TKZ_ERR_INVALID_JSON => error.InvalidJson,
        c.TKZ_ERR_MISSING_MODEL => error.MissingModel,
        c.TKZ_ERR_UNSUPPORTED_MODEL_TYPE => error.UnsupportedModelType,
        c.TKZ_ERR_MISSING_VOCAB => error.MissingVocab,
        c.TKZ_ERR_INVALID_VOCAB_ENTRY => error.InvalidVocabEntry,
        c.TKZ_ERR_OUT_OF_MEMORY => error.OutOfMemory,
        c.TKZ_ERR_FILE_NOT_FOUND => error.FileNotFound,
        c.TKZ_ERR_FILE_TOO_BIG => error.FileTooBig,
        c.TKZ_ERR_MISSING_UNK_TOKEN => error.MissingUnkToken,
        c.TKZ_ERR_INVALID_ARGUMENT => error.InvalidArgument,
        else => error.DeviceError,
    };
}

fn check(rc: c_int) Error!void {
    if (rc != c.TKZ_OK) return mapError(rc);
}

pub const GpuTokenizer = struct {
    h: *c.tkz_tokenizer,
    allocator: std.mem.Allocator,
    /// Tokenizer.truncation / .padding (lib.zig:41-42): set through setTruncation /
    /// setPadding so the device applies them (Tokenizer.encode steps 6-7).
    truncation: ?TruncationParams = null,
    padding: ?PaddingParams = null,

    const Self = @This();

    /// Tokenizer.fromFile (lib.zig:48-56): 100-MiB cap -> error.FileTooBig.
    pub fn fromFile(allocator: std.mem.Allocator, path: []const u8) Error!Self {
        const z = allocator.dupeZ(u8, path) catch return error.OutOfMemory;
        defer allocator.free(z);
        var h: ?*c.tkz_tokenizer = null;
        try check(c.tkz_create_from_file(z.ptr, &h));
        return .{ .h = h.?, .allocator = allocator };
    }

    /// Tokenizer.fromJson (lib.zig:59-85): loadConfig + added tokens.
    pub fn fromJson(allocator: std.mem.Allocator, json_content: []const u8) Error!Self {
        var h: ?*c.tkz_tokenizer = null;
        try check(c.tkz_create_from_json(json_content.ptr, json_content.len, &h));
        return .{ .h = h.?, .allocator = allocator };
    }

    /// Tokenizer.deinit (lib.zig:87-106).
    pub fn deinit(self: *Self) void {
        c.tkz_destroy(self.h);
    }

    /// Tokenizer.encode (lib.zig:109-160), computed on the GPU: the same Encoding
    /// (ids, type_ids, tokens, pretoken-relative offsets, masks), caller-owned.
    pub fn encode(self: *Self, text: []const u8, add_special_tokens: bool) Error!Encoding {
        var e: c.tkz_encoding = undefined;
        try check(c.tkz_encode(self.h, text.ptr, text.len, @intFromBool(add_special_tokens), &e));
        defer c.tkz_encoding_free(&e);
        const n = e.len;
        const a = self.allocator;
        var enc = Encoding{
            .allocator = a,
            .ids = a.dupe(u32, e.ids[0..n]) catch return error.OutOfMemory,
            .type_ids = a.dupe(u32, e.type_ids[0..n]) catch return error.OutOfMemory,
            .tokens = a.alloc([]const u8, n) catch return error.OutOfMemory,
            .offsets = a.alloc(Offset, n) catch return error.OutOfMemory,
            .special_token_mask = a.dupe(u32, e.special_token_mask[0..n]) catch return error.OutOfMemory,
            .attention_mask = a.dupe(u32, e.attention_mask[0..n]) catch return error.OutOfMemory,
            .words = null,
            .overflowing = &.{},
            .owns_token_strs = true,
        };
        for (0..n) |i| {
            enc.tokens[i] = a.dupe(u8, e.tokens[i][0..e.token_lens[i]]) catch return error.OutOfMemory;
            enc.offsets[i] = .{ .start = e.offsets[i].start, .end = e.offsets[i].end };
        }
        return enc;
    }

    /// Tokenizer.decode (lib.zig:163-189) + the config decoder; caller-owned bytes.
    pub fn decode(self: *Self, ids: []const u32, skip_special_tokens: bool) Error![]u8 {
        var out: [*c]u8 = null;
        var len: usize = 0;
        try check(c.tkz_decode(self.h, ids.ptr, ids.len, @intFromBool(skip_special_tokens), &out, &len));
        defer c.tkz_string_free(out);
        return self.allocator.dupe(u8, out[0..len]) catch error.OutOfMemory;
    }

    /// Tokenizer.addSpecialTokens (lib.zig:192-200): the number newly added.
    pub fn addSpecialTokens(self: *Self, tokens: []const AddedToken) Error!usize {
        const a = self.allocator;
        const ptrs = a.alloc([*c]const u8, tokens.len) catch return error.OutOfMemory;
        defer a.free(ptrs);
        const lens = a.alloc(usize, tokens.len) catch return error.OutOfMemory;
        defer a.free(lens);
        const ids = a.alloc(u32, tokens.len) catch return error.OutOfMemory;
        defer a.free(ids);
        for (tokens, 0..) |t, i| {
            ptrs[i] = t.content.ptr;
            lens[i] = t.content.len;
            ids[i] = t.id orelse c.TKZ_NO_ID;
        }
        return c.tkz_add_special_tokens_ids(self.h, ptrs.ptr, lens.ptr, ids.ptr, tokens.len);
    }

    /// Tokenizer.getVocabSize (lib.zig:203-205): model vocab + added tokens.
    pub fn getVocabSize(self: *const Self) usize {
        return c.tkz_get_vocab_size(self.h);
    }

    /// Tokenizer.tokenToId (lib.zig:208-214): the added vocab first, then the model's.
    pub fn tokenToId(self: *const Self, token: []const u8) ?u32 {
        var id: u32 = 0;
        return if (c.tkz_token_to_id(self.h, token.ptr, token.len, &id) != 0) id else null;
    }

    /// Tokenizer.idToToken (lib.zig:217-223): borrowed, valid until deinit.
    pub fn idToToken(self: *const Self, id: u32) ?[]const u8 {
        var len: usize = 0;
        const p = c.tkz_id_to_token(self.h, id, &len);
        return if (p == null) null else p[0..len];
    }

    /// Setting Tokenizer.truncation (lib.zig:41, applied at lib.zig:150-152).
    pub fn setTruncation(self: *Self, t: ?TruncationParams) Error!void {
        self.truncation = t;
        if (t) |p| {
            try check(c.tkz_set_truncation(self.h, 1, p.max_length, p.stride));
        } else try check(c.tkz_set_truncation(self.h, 0, 0, 0));
    }

    /// Setting Tokenizer.padding (lib.zig:42, applied at lib.zig:154-157).
    pub fn setPadding(self: *Self, p: ?PaddingParams) Error!void {
        self.padding = p;
        if (p) |q| {
            // PaddingParams.length null: nothing to pad to (encoding.zig:385-390)
            try check(c.tkz_set_padding(self.h, 1, q.length orelse 0, q.pad_id, q.pad_type_id, q.pad_token.ptr,
                q.pad_token.len, @intFromBool(q.direction == .left)));
        } else try check(c.tkz_set_padding(self.h, 0, 0, 0, 0, null, 0, 0));
    }

    // ---- batch API (no reference counterpart: the reference encodes one doc per call) ----

    /// Every doc of bytes[doc_off[i]..doc_off[i+1]] encoded as Tokenizer.encode would, as
    /// CSR (row_ptr, ids, offsets); free with freeBatch.
    pub fn encodeBatch(self: *Self, bytes: []const u8, doc_off: []const u64) Error!c.tkz_batch {
        var out: c.tkz_batch = undefined;
        try check(c.tkz_encode_batch(self.h, bytes.ptr, doc_off.ptr, doc_off.len - 1, &out));
        return out;
    }

    /// encodeBatch over several GPUs of this process (bit i of gpu_mask = device i).
    pub fn encodeBatchGpus(self: *Self, bytes: []const u8, doc_off: []const u64, gpu_mask: u32) Error!c.tkz_batch {
        var out: c.tkz_batch = undefined;
        try check(c.tkz_encode_batch_gpus(self.h, bytes.ptr, doc_off.ptr, doc_off.len - 1, gpu_mask, &out));
        return out;
    }

    pub fn freeBatch(_: *Self, b: *c.tkz_batch) void {
        c.tkz_batch_free(b);
    }

    /// Decodes every row of a CSR batch on the GPU; free with freeTextBatch.
    pub fn decodeBatch(self: *Self, row_ptr: []const u64, ids: []const u32, skip_special_tokens: bool) Error!c.tkz_text_batch {
        var out: c.tkz_text_batch = undefined;
        try check(c.tkz_decode_batch(self.h, row_ptr.ptr, ids.ptr, row_ptr.len - 1, @intFromBool(skip_special_tokens), &out));
        return out;
    }

    pub fn freeTextBatch(_: *Self, b: *c.tkz_text_batch) void {
        c.tkz_text_batch_free(b);
    }

    /// FastTokenizer.encode (lib.zig:352-413) over a batch: row d = the SpanEncoding of
    /// doc d (same caps); free with c.tkz_span_batch_free.
    pub fn fastEncodeBatch(self: *Self, bytes: []const u8, doc_off: []const u64, opts: c.tkz_fast_options) Error!c.tkz_span_batch {
        var out: c.tkz_span_batch = undefined;
        try check(c.tkz_fast_encode_batch(self.h, bytes.ptr, doc_off.ptr, doc_off.len - 1, &opts, &out));
        return out;
    }

    /// Page-locked host memory for batch input text (tkz_host_alloc): encodeBatch copies it
    /// to the device at the full PCIe rate. Any []const u8 works; this one is faster.
    pub fn allocInput(_: *Self, n: usize) Error![]u8 {
        const p = c.tkz_host_alloc(n) orelse return error.OutOfMemory;
        return @as([*]u8, @ptrCast(p))[0..n];
    }
    pub fn freeInput(_: *Self, buf: []u8) void {
        c.tkz_host_free(buf.ptr);
    }

    /// Tuning switches that never change a result (tkz.h): the BPE word memo and the
    /// segmented path of long pretokens (whole-text pre_tokenizers, config.zig:387-402).
    pub fn setWordMemo(self: *Self, on: bool) Error!void {
        try check(c.tkz_set_word_memo(self.h, @intFromBool(on)));
    }
    pub fn setLongSegments(self: *Self, on: bool) Error!void {
        try check(c.tkz_set_long_segments(self.h, @intFromBool(on)));
    }
};

test "GpuTokenizer mirrors Tokenizer (lib.zig:749-805 vector)" {
    const json =
        \\{"model":{"type":"WordPiece","vocab":{"[PAD]":0,"[UNK]":1,"[CLS]":2,"[SEP]":3,"hello":4,
        \\"world":5,"test":6,",":7,".":8,"!":9}},"normalizer":{"type":"BertNormalizer"},
        \\"pre_tokenizer":{"type":"BertPreTokenizer"}}
    ;
    var t = try GpuTokenizer.fromJson(std.testing.allocator, json);
    defer t.deinit();
    try std.testing.expectEqual(@as(usize, 10), t.getVocabSize());
    try std.testing.expectEqual(@as(?u32, 4), t.tokenToId("hello"));
    var enc = try t.encode("Hello, World!", true);
    defer enc.deinit();
    try std.testing.expectEqualSlices(u32, &.{ 4, 7, 5, 9 }, enc.ids);
}
