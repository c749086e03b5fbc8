"""Keyed counter RNG — Python twin of js/keyed-rng.mjs, used by the host to
build World.cloudNoise.p deterministically (js/noise.js:6-18) and by tests."""
import math

M32 = 0xFFFFFFFF
PERM_STREAM = 0xFFFFFFFF


def lowbias32(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def seed_mix(seed):
    return lowbias32((seed ^ 0x3C6EF372) & M32)


def sample_key(seedm, pixel, sample):
    return lowbias32(lowbias32((seedm ^ pixel) & M32) ^ lowbias32((sample + 0x1B873593) & M32))


def draw(skey, k):
    return (lowbias32(skey ^ ((k * 0x9E3779B9) & M32)) >> 8) * (1.0 / 16777216.0)


class KeyedStream:
    def __init__(self, seed):
        self.seedm = seed_mix(seed)
        self.key = 0
        self.k = 0

    def select(self, pixel, sample):
        self.key = sample_key(self.seedm, pixel & M32, sample & M32)
        self.k = 0

    def next(self):
        r = draw(self.key, self.k)
        self.k += 1
        return r


def permutation(seed):
    """PerlinNoise.p exactly as js/noise.js:6-18 shuffles it, from the keyed perm stream."""
    st = KeyedStream(seed)
    st.select(PERM_STREAM, PERM_STREAM)
    p = list(range(256))
    for i in range(255, -1, -1):
        j = math.floor(st.next() * (i + 1))
        p[i], p[j] = p[j], p[i]
    return p + p
