"""Pure-Python secp256k1 oracle (affine arithmetic, Python big ints).

Used only by the tests to check the native CPU implementation
(csrc/secp256k1/secp256k1.cpp) and the GPU batch verifier
(csrc/kernels/secp256k1.hip). Slow but obviously correct: every group
operation is the textbook affine formula.
"""
from __future__ import annotations

import hashlib
import hmac

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (
    0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
    0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8,
)


def point_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return (x, (lam * (a[0] - x) - a[1]) % P)


def point_mul(k, pt=G):
    r = None
    k %= N
    while k:
        if k & 1:
            r = point_add(r, pt)
        pt = point_add(pt, pt)
        k >>= 1
    return r


def serialize_pubkey(pt, compressed=True) -> bytes:
    x = pt[0].to_bytes(32, "big")
    if compressed:
        return bytes([2 + (pt[1] & 1)]) + x
    return b"\x04" + x + pt[1].to_bytes(32, "big")


def parse_pubkey(b: bytes):
    if len(b) == 33 and b[0] in (2, 3):
        x = int.from_bytes(b[1:], "big")
        if x >= P:
            return None
        y2 = (pow(x, 3, P) + 7) % P
        y = pow(y2, (P + 1) // 4, P)
        if y * y % P != y2:
            return None
        if (y & 1) != (b[0] & 1):
            y = P - y
        return (x, y)
    if len(b) == 65 and b[0] in (4, 6, 7):
        x = int.from_bytes(b[1:33], "big")
        y = int.from_bytes(b[33:], "big")
        if x >= P or y >= P or (y * y - x * x * x - 7) % P:
            return None
        if b[0] in (6, 7) and (y & 1) != (b[0] & 1):
            return None
        return (x, y)
    return None


def pubkey_from_secret(sec: bytes, compressed=True) -> bytes:
    return serialize_pubkey(point_mul(int.from_bytes(sec, "big")), compressed)


def rfc6979_nonce(msg32: bytes, key32: bytes, extra32: bytes | None = None, counter: int = 0) -> bytes:
    """libsecp256k1 nonce_function_rfc6979: HMAC-DRBG seeded with key || msg [|| extra]."""
    seed = key32 + msg32 + (extra32 or b"")
    v = b"\x01" * 32
    k = b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + seed, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + seed, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    out = b""
    for _ in range(counter + 1):
        while True:
            v = hmac.new(k, v, hashlib.sha256).digest()
            t = int.from_bytes(v, "big")
            if 0 < t < N:
                out = v
                break
            k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
            v = hmac.new(k, v, hashlib.sha256).digest()
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()
    return out


def sign(sec: bytes, msg32: bytes, extra32: bytes | None = None):
    """Returns (r, s, recid) with low-S normalisation."""
    d = int.from_bytes(sec, "big")
    z = int.from_bytes(msg32, "big") % N
    counter = 0
    while True:
        k = int.from_bytes(rfc6979_nonce(msg32, sec, extra32, counter), "big")
        R = point_mul(k)
        r = R[0] % N
        recid = (R[1] & 1) | (2 if R[0] >= N else 0)
        s = pow(k, -1, N) * (z + r * d) % N
        if r and s:
            break
        counter += 1
    if s > N // 2:
        s = N - s
        recid ^= 1
    return r, s, recid


def der_encode(r: int, s: int) -> bytes:
    def enc(v):
        b = v.to_bytes(33, "big").lstrip(b"\x00")
        if not b or b[0] & 0x80:
            b = b"\x00" + b
        return b"\x02" + bytes([len(b)]) + b

    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


def der_decode(sig: bytes):
    """(r, s) of a strict DER signature (as produced by der_encode / the node's signer)."""
    if len(sig) < 8 or sig[0] != 0x30 or sig[2] != 0x02:
        raise ValueError("not a DER signature")
    lr = sig[3]
    r = int.from_bytes(sig[4:4 + lr], "big")
    off = 4 + lr
    if sig[off] != 0x02:
        raise ValueError("not a DER signature")
    ls = sig[off + 1]
    return r, int.from_bytes(sig[off + 2:off + 2 + ls], "big")


def verify(pub: bytes, r: int, s: int, msg32: bytes, require_low_s=True) -> bool:
    Q = parse_pubkey(pub)
    if Q is None or not (0 < r < N and 0 < s < N):
        return False
    if require_low_s and s > N // 2:
        return False
    z = int.from_bytes(msg32, "big") % N
    w = pow(s, -1, N)
    X = point_add(point_mul(z * w % N), point_mul(r * w % N, Q))
    return X is not None and X[0] % N == r


def recover(r: int, s: int, recid: int, msg32: bytes):
    x = r + (N if recid & 2 else 0)
    if x >= P:
        return None
    y2 = (pow(x, 3, P) + 7) % P
    y = pow(y2, (P + 1) // 4, P)
    if y * y % P != y2:
        return None
    if (y & 1) != (recid & 1):
        y = P - y
    R = (x, y)
    z = int.from_bytes(msg32, "big") % N
    rinv = pow(r, -1, N)
    return point_add(point_mul(s * rinv % N, R), point_mul((-z * rinv) % N))
