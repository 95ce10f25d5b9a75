"""rand 0.8 `StdRng` restated: ChaCha12 keystream + rand_core 0.6 `seed_from_u64`.

The reference samples which constraint elements are active with
`StdRng::seed_from_u64(3019)` and `rng.gen::<f64>() <= proportion`
(src/viterbi_solver/utils.rs:101 and 168-177).  rand 0.8's StdRng is rand_chacha 0.3's
ChaCha12Rng; these crates are not vendored in the reference (Cargo.toml:14, no lockfile),
so this follows their published algorithms:

* rand_core 0.6 `SeedableRng::seed_from_u64`: a PCG32 step per 4-byte chunk of the 32-byte
  seed (state = state * 6364136223846793005 + 11634580027462260723; output
  rotr32(((state >> 18) ^ state) >> 27, state >> 59), little endian).
* rand_chacha 0.3 ChaCha12Rng::from_seed: key = seed, 64-bit block counter from 0, 64-bit
  stream id 0 (djb ChaCha layout), 6 double rounds; blocks are emitted in counter order.
* rand_core BlockRng::next_u64 = lo word | hi word << 32 of two consecutive u32 outputs.
* rand 0.8 `Standard` f64 = (next_u64 >> 11) * 2^-53.

The ChaCha core is checked against the published all-zero-key ChaCha20 keystream
(tests/test_host.py); the seeding and the f64 conversion are pinned by the crates' source
as restated above only ("parity unpinned" -- no Rust toolchain here to run the reference).
"""
from __future__ import annotations

import numpy as np

_M32 = 0xFFFFFFFF


def _rotl(x, n):
    return ((x << np.uint32(n)) | (x >> np.uint32(32 - n))) & np.uint32(_M32)


def chacha_blocks(key_words, counter0, nblocks, rounds=12, stream=0):
    """nblocks ChaCha blocks (16 u32 each) for counters counter0.. ; djb 64-bit counter/nonce."""
    with np.errstate(over="ignore"):
        ctr = np.arange(counter0, counter0 + nblocks, dtype=np.uint64)
        st = np.zeros((nblocks, 16), np.uint32)
        st[:, 0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], np.uint32)
        st[:, 4:12] = np.asarray(key_words, np.uint32)
        st[:, 12] = (ctr & np.uint64(_M32)).astype(np.uint32)
        st[:, 13] = (ctr >> np.uint64(32)).astype(np.uint32)
        st[:, 14] = np.uint32(stream & _M32)
        st[:, 15] = np.uint32(stream >> 32)
        x = st.copy()

        def qr(a, b, c, d):
            x[:, a] += x[:, b]
            x[:, d] = _rotl(x[:, d] ^ x[:, a], 16)
            x[:, c] += x[:, d]
            x[:, b] = _rotl(x[:, b] ^ x[:, c], 12)
            x[:, a] += x[:, b]
            x[:, d] = _rotl(x[:, d] ^ x[:, a], 8)
            x[:, c] += x[:, d]
            x[:, b] = _rotl(x[:, b] ^ x[:, c], 7)

        for _ in range(rounds // 2):
            qr(0, 4, 8, 12)
            qr(1, 5, 9, 13)
            qr(2, 6, 10, 14)
            qr(3, 7, 11, 15)
            qr(0, 5, 10, 15)
            qr(1, 6, 11, 12)
            qr(2, 7, 8, 13)
            qr(3, 4, 9, 14)
        return x + st


def seed_from_u64(state: int):
    """rand_core 0.6 SeedableRng::seed_from_u64 -> 8 little-endian key words."""
    mul, inc = 6364136223846793005, 11634580027462260723
    words = []
    for _ in range(8):
        state = (state * mul + inc) & 0xFFFFFFFFFFFFFFFF
        xorshifted = (((state >> 18) ^ state) >> 27) & _M32
        rot = state >> 59
        words.append(((xorshifted >> rot) | (xorshifted << ((-rot) & 31))) & _M32)
    return words


class StdRng:
    """rand 0.8 StdRng (ChaCha12Rng) with seed_from_u64; only what the reference uses."""

    def __init__(self, seed: int):
        self.key = seed_from_u64(seed)
        self.counter = 0  # next block counter
        self.buf = np.zeros(0, np.uint32)
        self.idx = 0

    def _refill(self):
        # rand_chacha fills 4 blocks (64 words) at a time; the word stream is block order
        self.buf = chacha_blocks(self.key, self.counter, 4).reshape(-1)
        self.counter += 4
        self.idx = 0

    def next_u64_array(self, n: int) -> np.ndarray:
        """n successive next_u64() values (only u64 draws are made, so index stays even)."""
        out = np.empty(n, np.uint64)
        k = 0
        while k < n:
            if self.idx >= len(self.buf):
                self._refill()
            take = min((len(self.buf) - self.idx) // 2, n - k)
            w = self.buf[self.idx:self.idx + 2 * take].astype(np.uint64)
            out[k:k + take] = w[0::2] | (w[1::2] << np.uint64(32))
            self.idx += 2 * take
            k += take
        return out

    def gen_f64(self, n: int) -> np.ndarray:
        """n draws of rng.gen::<f64>(): (next_u64 >> 11) * 2^-53, in [0, 1)."""
        return (self.next_u64_array(n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
