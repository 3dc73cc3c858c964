"""64-bit rolling hashes of a CSR encode result (the C4 full-batch
check). h = h * M + x (mod 2^64) over the values in batch order, so a hash can be
continued block by block: the golden file is built from the oracle in blocks of docs,
the GPU result is hashed whole."""
import numpy as np

M = np.uint64(0x100000001B3)
H0 = 0xCBF29CE484222325


def roll(h: int, x: np.ndarray) -> int:
    """Continues hash h over the u64 values of x."""
    x = np.ascontiguousarray(x).astype(np.uint64, copy=False).ravel()
    hh = np.uint64(h)
    with np.errstate(over="ignore"):
        for s0 in range(0, len(x), 1 << 20):
            blk = x[s0:s0 + (1 << 20)]
            pw = np.cumprod(np.full(len(blk), M, dtype=np.uint64))  # M^1 .. M^n
            w = np.concatenate((np.ones(1, dtype=np.uint64), pw[:-1]))[::-1]  # M^(n-1) .. M^0
            hh = hh * pw[-1] + np.sum(blk * w, dtype=np.uint64)
    return int(hh)


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
