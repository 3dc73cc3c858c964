"""64-bit rolling hashes of a CSR encode result (the C4 full-batch
check). h = h * M + x (mod 2^64) over the values in batch order, so a hash can be
continued block by block: the golden file is built from the oracle in blocks of docs,
the GPU result is hashed whole."""
import numpy as np

M = np.uint64(0x100000001B3)
H0 = 0xCBF29CE484222325


BLK = 1 << 20
with np.errstate(over="ignore"):
    _PW = np.cumprod(np.full(BLK, M, dtype=np.uint64))  # M^1 .. M^BLK
    _W = np.concatenate((np.ones(1, dtype=np.uint64), _PW[:-1]))[::-1].copy()  # M^(BLK-1) .. M^0


def mpow(n: int) -> int:
    """M^n mod 2^64."""
    return pow(int(M), n, 1 << 64)


def roll(h: int, x: np.ndarray) -> int:
    """Continues hash h over the u64 values of x: h * M^n + sum(x_i * M^(n-1-i))."""
    x = np.ascontiguousarray(x).astype(np.uint64, copy=False).ravel()
    hh = np.uint64(h)
    with np.errstate(over="ignore"):
        for s0 in range(0, len(x), BLK):
            blk = x[s0:s0 + BLK]
            n = len(blk)
            hh = hh * _PW[n - 1] + np.sum(blk * _W[BLK - n:], dtype=np.uint64)
    return int(hh)


def geo(n: int) -> int:
    """sum(M^k, k < n) mod 2^64, by binary decomposition of n."""
    mod = 1 << 64
    total, power = 0, 1              # sum and M^(terms) of the prefix built so far
    blk_sum, blk_pow = 1, int(M)     # a block of 2^j terms: its sum and M^(2^j)
    while n:
        if n & 1:
            total = (total + power * blk_sum) % mod
            power = power * blk_pow % mod
        blk_sum = blk_sum * (1 + blk_pow) % mod
        blk_pow = blk_pow * blk_pow % mod
        n >>= 1
    return total


def combine(shards) -> dict:
    """Hashes of the concatenated batch from the per-shard results (each a CsrHash.result()
    of one shard's own CSR, in doc order): h_whole = h_whole * M^n + (h_shard - H0 * M^n),
    and the shard's row_ptr values are offset by the token base of the shards before it."""
    mod = 1 << 64
    h_row = roll(H0, np.zeros(1, np.uint64))
    h_ids = h_offs = H0
    base = n_tok = n_doc = 0
    for s in shards:
        nd, nt = s["n_docs"], s["n_tokens"]
        r_s, i_s, o_s = int(s["row_ptr"], 16), int(s["ids"], 16), int(s["offsets"], 16)
        # the shard's row hash starts with its row_ptr[0] = 0 term: h_s = roll(roll(H0, [0]), rows)
        h0r = roll(H0, np.zeros(1, np.uint64))
        z_row = (r_s - h0r * mpow(nd)) % mod
        h_row = (h_row * mpow(nd) + z_row + base * geo(nd)) % mod
        h_ids = (h_ids * mpow(nt) + (i_s - H0 * mpow(nt))) % mod
        h_offs = (h_offs * mpow(nt) + (o_s - H0 * mpow(nt))) % mod
        base += nt
        n_tok += nt
        n_doc += nd
    return {"n_docs": n_doc, "n_tokens": n_tok, "row_ptr": f"{h_row:016x}", "ids": f"{h_ids:016x}",
            "offsets": f"{h_offs:016x}"}


def offsets_u64(offs: np.ndarray) -> np.ndarray:
    """(T, 2) u32 offsets -> start | end << 32."""
    o = np.ascontiguousarray(offs, dtype=np.uint32)
    return o[:, 0].astype(np.uint64) | (o[:, 1].astype(np.uint64) << np.uint64(32))


class CsrHash:
    """Hashes of row_ptr, ids and offsets, fed in doc order (block by block)."""

    def __init__(self):
        self.h_row = roll(H0, np.zeros(1, np.uint64))  # row_ptr[0] = 0
        self.h_ids = H0
        self.h_offs = H0
        self.n_tokens = 0
        self.n_docs = 0

    def add(self, row: np.ndarray, ids: np.ndarray, offs: np.ndarray):
        """row: the block's local row_ptr (n + 1 entries, row[0] = 0)."""
        row = np.asarray(row, dtype=np.uint64)
        self.h_row = roll(self.h_row, row[1:] + np.uint64(self.n_tokens))
        self.h_ids = roll(self.h_ids, ids)
        self.h_offs = roll(self.h_offs, offsets_u64(offs))
        self.n_tokens += int(row[-1])
        self.n_docs += len(row) - 1

    def result(self) -> dict:
        return {"n_docs": self.n_docs, "n_tokens": self.n_tokens, "row_ptr": f"{self.h_row:016x}",
                "ids": f"{self.h_ids:016x}", "offsets": f"{self.h_offs:016x}"}
