"""Hash primitives vs hashlib/hmac and published vectors (reference src/test/crypto_tests.cpp)."""
import hashlib
import hmac
import os

import pytest


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 1000, 4096])
def test_sha2_family(native, n):
    d = os.urandom(n)
    assert native.sha256(d) == hashlib.sha256(d).digest()
    assert native.sha256d(d) == hashlib.sha256(hashlib.sha256(d).digest()).digest()
    assert native.sha512(d) == hashlib.sha512(d).digest()
    assert native.sha1(d) == hashlib.sha1(d).digest()


def test_ripemd160_vectors(native):
    assert native.ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"
    assert native.ripemd160(b"abc").hex() == "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"
    assert native.ripemd160(b"message digest").hex() == "5d0689ef49d2fae572b881b123a85ffa21595f36"
    assert native.ripemd160(b"a" * 1000000).hex() == "52783243c1697bdbe16d37f97f68f08325dc1528"


def test_hmac(native):
    for klen in (0, 20, 64, 65, 131):
        k = os.urandom(klen)
        d = os.urandom(77)
        assert native.hmac_sha256(k, d) == hmac.new(k, d, "sha256").digest()
        assert native.hmac_sha512(k, d) == hmac.new(k, d, "sha512").digest()


@pytest.mark.parametrize("n", [0, 1, 127, 128, 129, 140, 144, 255, 256, 257, 1000])
def test_blake2b_personal(native, n):
    d = os.urandom(n)
    person = b"ZcashPoW" + (200).to_bytes(4, "little") + (9).to_bytes(4, "little")
    assert native.blake2b(d, 50, person=person) == hashlib.blake2b(d, digest_size=50, person=person).digest()
    key, salt = os.urandom(33), os.urandom(16)
    assert native.blake2b(d, 64, key=key, salt=salt) == hashlib.blake2b(d, digest_size=64, key=key, salt=salt).digest()
    assert native.blake2b(d, 1) == hashlib.blake2b(d, digest_size=1).digest()


def test_siphash_vectors(native):
    # SipHash-2-4 reference vectors (key 00..0f, messages 00..n-1), as in reference hash_tests.cpp
    k0 = 0x0706050403020100
    k1 = 0x0F0E0D0C0B0A0908
    assert native.siphash(k0, k1, b"") == 0x726FDB47DD0E0E31
    assert native.siphash(k0, k1, bytes(range(1))) == 0x74F839C593DC67FD
    assert native.siphash(k0, k1, bytes(range(8))) == 0x93F5F5799A932462
    assert native.siphash(k0, k1, bytes(range(15))) == 0xA129CA6149BE45E5
    # uint256 fast paths agree with the streaming hasher
    v = os.urandom(32)
    assert native.siphash_uint256(k0, k1, v) == native.siphash(k0, k1, v)
    assert native.siphash_uint256_extra(k0, k1, v, 0x12345678) == native.siphash(
        k0, k1, v + (0x12345678).to_bytes(4, "little"))


def test_chacha20_vector(native):
    # RFC 7539 style all-zero key/iv keystream (reference crypto_tests.cpp chacha20 vectors)
    out = native.chacha20(bytes(32), 0, 0, 64)
    assert out.hex() == (
        "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
        "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def test_aes256cbc(native):
    key = bytes(range(32))
    ct = native.aes256cbc_encrypt(key, bytes(16), bytes.fromhex("00112233445566778899aabbccddeeff"), False)
    assert ct.hex() == "8ea2b7ca516745bfeafc49904b496089"  # FIPS-197 C.3
    for n in (0, 1, 15, 16, 17, 100):
        pt = os.urandom(n)
        iv = os.urandom(16)
        enc = native.aes256cbc_encrypt(key, iv, pt, True)
        if n:
            assert len(enc) % 16 == 0 and len(enc) > n
            assert native.aes256cbc_decrypt(key, iv, enc, True) == pt


def test_compact_bits(native):
    # reference arith_uint256_tests.cpp bignum_SetCompact
    assert native.compact_to_target_hex(0x1d00ffff)[0] == "00000000ffff" + "0" * 52
    assert native.compact_to_target_hex(0x01003456)[0] == "0" * 64
    t, neg, ovf = native.compact_to_target_hex(0x04923456)
    assert neg and t == "0" * 56 + "12345600"
    assert native.target_hex_to_compact("0" * 56 + "12345600", True) == 0x04923456
    assert native.compact_to_target_hex(0xff123456)[2]  # overflow
    assert native.target_hex_to_compact("00000000ffff" + "0" * 52) == 0x1d00ffff
    assert native.target_hex_to_compact("7fffff" + "0" * 58) == 0x207fffff
