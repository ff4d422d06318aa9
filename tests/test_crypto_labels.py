"""Primitive parity: CRT math, label codecs, fixed-key hash, PRG (reference
dash/test/test_util.h, test_label.h, test_cuda_aes_engine.h)."""
import numpy as np
import pytest

from tests.aes_ref import dash_hash, encrypt_block


def test_fips197_vector(native):
    k = bytes(range(16))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert native.aes_encrypt_block(k, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert encrypt_block(k, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_hash_matches_pure_python(native):
    rng = np.random.default_rng(7)
    for _ in range(20):
        x = int(rng.integers(0, 2**63)) | (int(rng.integers(0, 2**63)) << 64)
        assert native.aes_hash(x) == dash_hash(x)
    a = rng.integers(0, 2**63, size=(64, 2), dtype=np.uint64)
    h = native.aes_hash_array(a)
    for i in range(0, 64, 13):
        x = int(a[i, 0]) | (int(a[i, 1]) << 64)
        assert int(h[i, 0]) | (int(h[i, 1]) << 64) == dash_hash(x)


@pytest.mark.parametrize("p,n", [(2, 128), (3, 80), (5, 55), (7, 45), (11, 37), (13, 34), (17, 31), (19, 30),
                                 (23, 28), (32, 25), (97, 19), (167, 17)])
def test_label_width(native, p, n):
    assert native.nr_comps(p) == n


@pytest.mark.parametrize("p", [2, 3, 4, 5, 7, 8, 11, 13, 16, 17, 19, 23, 29, 31, 32, 56, 64, 86, 97, 107, 167, 173, 541])
def test_compress_roundtrip(native, p):
    rng = np.random.default_rng(p)
    n = native.nr_comps(p)
    for L in [np.zeros(n, np.int16), np.full(n, p - 1, np.int16), rng.integers(0, p, n).astype(np.int16)]:
        c = native.compress(L, p)
        assert c == sum(int(v) * p**i for i, v in enumerate(L)) % (1 << 128)
        np.testing.assert_array_equal(native.decompress(c, p), L)


def test_crt_and_primes(native):
    assert native.first_primes(8) == [2, 3, 5, 7, 11, 13, 17, 19]
    from dash_amd.ir.bases import first_primes

    assert first_primes(100)[-1] == 541
    assert native.mul_inv(3, 7) == 5
    assert native.mul_inv(2, 9) == 5


def test_crt_decode_reconstruction(native):
    # chinese remainder of 10000 over 8 primes (reference test_util.h:34)
    from dash_amd.ir.layers import Dense
    import dash_amd as d
    from dash_amd.garbling import GarbledCircuit

    c = d.Circuit([Dense.from_quantized(np.eye(3, dtype=np.int64), np.zeros(3, np.int64))])
    gc = GarbledCircuit(c, 8, None, seed=bytes(16))
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs([10000, -10000, 4849844])))
    np.testing.assert_array_equal(out, [10000, -10000, 4849844])


def test_prg_deterministic(native):
    a = native.prg_label(bytes(16), 5, 0, 17)
    b = native.prg_label(bytes(16), 5, 0, 17)
    c = native.prg_label(bytes(16), 6, 0, 17)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, c)
    assert a.min() >= 0 and a.max() < 17


@pytest.mark.parametrize("p", [2, 3, 7, 17, 32, 64, 86, 97, 173])
def test_prg_label_matches_oracle(native, p):
    """Prg::label (core.h): block b = AES_seed(stream || ctr + b) (little-endian 128-bit) supplies components
    b*m .. b*m + m - 1 as its least significant base-p digits, m = largest count with p^m <= 2^64 (all
    128 / log2 p bits for powers of two). Pure-Python oracle on tests/aes_ref.py."""
    seed, stream, ctr = bytes(range(3, 19)), 0x1234_5678_9ABC, 41
    n = native.nr_comps(p)
    if p & (p - 1) == 0:
        m = 128 // (p.bit_length() - 1)
    else:
        m = 0
        while p ** (m + 1) <= 2 ** 64:
            m += 1
    exp = []
    b = 0
    while len(exp) < n:
        blk = ((stream << 64) | (ctr + b)).to_bytes(16, "little")
        v = int.from_bytes(encrypt_block(seed, blk), "little")
        for _ in range(min(m, n - len(exp))):
            exp.append(v % p)
            v //= p
        b += 1
    np.testing.assert_array_equal(native.prg_label(seed, stream, ctr, p), exp)
