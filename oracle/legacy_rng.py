"""Pure-Python restatement of NumPy's legacy ``RandomState`` stream (SURVEY.md
Appendix B) -- TEST INFRASTRUCTURE ONLY (checker for the device MT19937).

NumPy sources restated (numpy/random, stream frozen by NumPy's compatibility policy):
* ``mt19937_seed``   -- ``np.random.seed(s)`` for integer s: init_genrand(s)
* ``mt19937_gen``    -- the 624-word twist; ``mt19937_next`` -- tempering
* ``legacy_double``  -- 53-bit double from two draws: (a>>5, b>>6)
* ``legacy_gauss``   -- polar Box-Muller with one cached deviate
* ``buffered_bounded_masked_uint32`` -- ``randint(0, n)`` by masked rejection

The sampler consumes, per iteration: randint (apf_step2.py:302), one gauss inside
proposal/logproposal (:64/:68), one rand in accept_reject (:143).
"""
from __future__ import annotations

import math

N, M = 624, 397
MATRIX_A = 0x9908B0DF
UPPER, LOWER = 0x80000000, 0x7FFFFFFF


class LegacyMT:
    def __init__(self, seed: int):
        seed &= 0xFFFFFFFF
        key = [0] * N
        for pos in range(N):
            key[pos] = seed
            seed = (1812433253 * (seed ^ (seed >> 30)) + pos + 1) & 0xFFFFFFFF
        self.key = key
        self.pos = N
        self.has_gauss = False
        self.gauss_cache = 0.0

    def _twist(self):
        k = self.key
        for i in range(N - M):
            y = (k[i] & UPPER) | (k[i + 1] & LOWER)
            k[i] = k[i + M] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
        for i in range(N - M, N - 1):
            y = (k[i] & UPPER) | (k[i + 1] & LOWER)
            k[i] = k[i + (M - N)] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
        y = (k[N - 1] & UPPER) | (k[0] & LOWER)
        k[N - 1] = k[M - 1] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
        self.pos = 0

    def next_u32(self) -> int:
        if self.pos == N:
            self._twist()
        y = self.key[self.pos]
        self.pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def rand(self) -> float:
        a = self.next_u32() >> 5
        b = self.next_u32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0

    def gauss(self) -> float:
        if self.has_gauss:
            self.has_gauss = False
            v = self.gauss_cache
            self.gauss_cache = 0.0
            return v
        while True:
            x1 = 2.0 * self.rand() - 1.0
            x2 = 2.0 * self.rand() - 1.0
            r2 = x1 * x1 + x2 * x2
            if r2 < 1.0 and r2 != 0.0:
                break
        f = math.sqrt(-2.0 * math.log(r2) / r2)
        self.gauss_cache = f * x1
        self.has_gauss = True
        return f * x2

    def randint(self, n: int) -> int:
        """``randint(0, n)``: masked rejection with the smallest all-ones mask >= n-1."""
        rng = n - 1
        mask = rng
        for s in (1, 2, 4, 8, 16):
            mask |= mask >> s
        while True:
            v = self.next_u32() & mask
            if v <= rng:
                return v

    def state(self):
        """(key[624], pos, has_gauss, gauss) -- the layout olpe_rng_get/set use."""
        return list(self.key), self.pos, self.has_gauss, self.gauss_cache
