"""Independent pure-Python AES-128 (FIPS-197) used to cross-check the native
AES-NI and HIP T-table implementations (wire-compatibility vectors)."""


def _xt(a):
    return ((a << 1) ^ 0x1B) & 0xFF if a & 0x80 else a << 1


def _gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xt(a)
        b >>= 1
    return r


SBOX = []
for x in range(256):
    inv = next((y for y in range(1, 256) if _gmul(x, y) == 1), 0) if x else 0
    s = inv
    for i in range(1, 5):
        s ^= ((inv << i) | (inv >> (8 - i))) & 0xFF
    SBOX.append(s ^ 0x63)


def expand_key(key: bytes):
    rcon = [1, 2, 4, 8, 16, 32, 64, 128, 27, 54]
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [SBOX[b] for b in t[1:] + t[:1]]
            t[0] ^= rcon[i // 4 - 1]
        w.append([a ^ b for a, b in zip(w[i - 4], t)])
    return [sum(w[4 * r:4 * r + 4], []) for r in range(11)]


def encrypt_block(key: bytes, block: bytes) -> bytes:
    rk = expand_key(key)
    s = [b ^ k for b, k in zip(block, rk[0])]
    for r in range(1, 11):
        s = [SBOX[b] for b in s]
        s = [s[(i + 4 * (i % 4)) % 16] for i in range(16)]  # ShiftRows (column-major state)
        if r < 10:
            out = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                out += [_gmul(a[0], 2) ^ _gmul(a[1], 3) ^ a[2] ^ a[3], a[0] ^ _gmul(a[1], 2) ^ _gmul(a[2], 3) ^ a[3],
                        a[0] ^ a[1] ^ _gmul(a[2], 2) ^ _gmul(a[3], 3), _gmul(a[0], 3) ^ a[1] ^ a[2] ^ _gmul(a[3], 2)]
            s = out
        s = [b ^ k for b, k in zip(s, rk[r])]
    return bytes(s)


def dash_hash(x: int) -> int:
    """H(C) = AES-128_{00..0f}(LE bytes of C) as a little-endian 128-bit int."""
    return int.from_bytes(encrypt_block(bytes(range(16)), x.to_bytes(16, "little")), "little")
