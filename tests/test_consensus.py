"""Consensus data model, difficulty, merkle, secp256k1, keys and address encodings.

Golden values come from the reference's own unit tests (cited per test) and from
independent Python oracles (hashlib, bitcoincashplus_amd.utils.secp256k1_ref).
Reference JSON vectors are vendored as plain JSON under tests/data/vectors/.
"""
import hashlib
import json
import os
import random

import pytest

from bitcoincashplus_amd.utils import secp256k1_ref as ref

REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "vectors")  # vendored from reference src/test/data


def sha256d(b):
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def load_ref_json(name):
    path = os.path.join(REF_DATA, name)
    if not os.path.exists(path):
        pytest.skip(f"reference vectors not mounted: {path}")
    with open(path) as f:
        return json.load(f)


# ------------------------------------------------------------------ chain params
def test_genesis_hashes(native):
    # reference src/chainparams.cpp asserts
    assert native.chain_params("main")["genesis_hash"] == \
        "000000000019d6689c085ae165831e934ff763ae46a2a6c172b3f1b60a8ce26f"
    assert native.chain_params("test")["genesis_hash"] == \
        "000000000933ea01ad0ee984209779baaec3ced90fa3f408719526f8d77f4943"
    assert native.chain_params("regtest")["genesis_hash"] == \
        "0f9188f13cb7b2c71f2a335e3a4fc328bf5beb436012afca590b1a11466e2206"
    for c in ("main", "test", "regtest"):
        assert native.chain_params(c)["genesis_merkle_root"] == \
            "4a5e1e4baab89f3a32518a88c31bc87f618f76673e2cc77ab2127b7afdeda33b"


def test_chain_params_equihash(native):
    assert (native.chain_params("main")["equihash_n"], native.chain_params("main")["equihash_k"]) == (200, 9)
    assert (native.chain_params("regtest")["equihash_n"], native.chain_params("regtest")["equihash_k"]) == (48, 5)
    assert native.chain_params("regtest")["bcp_height"] == 3000
    assert native.chain_params("main")["cashaddr_prefix"] == "bitcoincashplus"
    assert native.chain_params("test")["cashaddr_prefix"] == "bcptest"
    assert native.chain_params("regtest")["cashaddr_prefix"] == "bcpreg"


def test_genesis_block_roundtrip(native):
    raw = native.genesis_block("main")
    d = native.block_decode(raw, legacy=True, chain="main")
    assert d["hash"] == native.chain_params("main")["genesis_hash"]
    assert d["computed_merkle_root"] == d["merkle_root"]
    assert not d["mutated"]
    assert d["reserialized"] == raw
    # legacy header hash == sha256d of the 80-byte header
    assert sha256d(raw[:80])[::-1].hex() == d["hash"]


def test_block_subsidy(native):
    assert native.block_subsidy(0, "main") == 50 * 100_000_000
    assert native.block_subsidy(210000, "main") == 25 * 100_000_000
    assert native.block_subsidy(64 * 210000, "main") == 0


# ------------------------------------------------------------------ difficulty
def test_get_next_work_legacy(native):
    # reference src/test/pow_tests.cpp:18-75
    assert native.calculate_next_work(32255, 1262152739, 0x1d00ffff, 1261130161, "main") == 0x1d00d86a
    assert native.calculate_next_work(2015, 1233061996, 0x1d00ffff, 1231006505, "main") == 0x1d00ffff
    assert native.calculate_next_work(68543, 1279297671, 0x1c05a3f4, 1279008237, "main") == 0x1c0168fd
    assert native.calculate_next_work(46367, 1269211443, 0x1c387f6f, 1263163443, "main") == 0x1d00e1fd


def _target(bits):
    exp = bits >> 24
    mant = bits & 0x7FFFFF
    return mant << (8 * (exp - 3)) if exp > 3 else mant >> (8 * (3 - exp))


def test_cash_plus_difficulty(native):
    # reference src/test/pow_tests.cpp:114-290 (golden nBits)
    p = native.chain_params("main")
    pow_limit = int(p["pow_limit_legacy"], 16)
    sim = native.ChainSim("main")

    def compact(v):
        size = (v.bit_length() + 7) // 8
        if size <= 3:
            c = v << (8 * (3 - size))
        else:
            c = v >> (8 * (size - 3))
        if c & 0x00800000:
            c >>= 8
            size += 1
        return c | (size << 24)

    initial = compact(pow_limit >> 4)
    sim.add(1269211443, initial, absolute=True)
    for _ in range(1, 2050):
        sim.add(600, initial)
    bits = sim.cashplus_next_work()
    for _ in range(10):
        sim.add(600, bits)
        assert sim.cashplus_next_work() == bits
    sim.add(6000, bits)
    assert sim.cashplus_next_work() == bits
    sim.add(2 * 600 - 6000, bits)
    assert sim.cashplus_next_work() == bits
    for _ in range(20):
        sim.add(600, bits)
        assert sim.cashplus_next_work() == bits
    sim.add(550, bits)
    assert sim.cashplus_next_work() == bits
    for _ in range(10):
        sim.add(550, bits)
        nb = sim.cashplus_next_work()
        assert _target(nb) < _target(bits)
        assert _target(bits) - _target(nb) < _target(bits) >> 10
        bits = nb
    assert bits == 0x1c0fe7b1
    for _ in range(20):
        sim.add(10, bits)
        nb = sim.cashplus_next_work()
        assert _target(nb) < _target(bits)
        bits = nb
    assert bits == 0x1c0db19f
    sim.add(6000, bits)
    bits = sim.cashplus_next_work()
    assert bits == 0x1c0d9222
    for _ in range(93):
        sim.add(6000, bits)
        nb = sim.cashplus_next_work()
        assert _target(nb) > _target(bits)
        assert _target(nb) <= pow_limit
        bits = nb
    assert bits == 0x1c2f13b9
    sim.add(6000, bits)
    bits = sim.cashplus_next_work()
    assert bits == 0x1c2ee9bf
    for _ in range(192):
        sim.add(6000, bits)
        nb = sim.cashplus_next_work()
        assert _target(nb) > _target(bits)
        bits = nb
    assert bits == 0x1d00ffff
    for _ in range(5):
        sim.add(6000, bits)
        assert sim.cashplus_next_work() == 0x1d00ffff


def test_fork_difficulty_windows(native):
    # Premine window -> powLimit(postfork); averaging window -> powLimitStart
    # (reference src/pow.cpp:71-100).
    p = native.chain_params("test")
    sim = native.ChainSim("test")
    fork = p["bcp_height"]
    sim.start_height = fork - 3
    t = 1500000000
    sim.add(t, 0x1d00ffff, absolute=True)
    sim.add(600, 0x1d00ffff)
    # next block is fork - 1 -> legacy rule (testnet min-difficulty off for this time)
    assert sim.height == fork - 2
    sim.add(600, 0x1d00ffff)
    # next height == fork: premine window
    bits = sim.next_work(t + 1800)
    assert bits == _compact_hex(p["pow_limit"])


def _compact_hex(h):
    v = int(h, 16)
    size = (v.bit_length() + 7) // 8
    c = v >> (8 * (size - 3)) if size > 3 else v << (8 * (3 - size))
    if c & 0x00800000:
        c >>= 8
        size += 1
    return c | (size << 24)


def test_check_proof_of_work(native):
    g = native.chain_params("main")["genesis_hash"]
    assert native.check_proof_of_work(g, 0x1d00ffff, False, "main")
    assert not native.check_proof_of_work("f" * 64, 0x1d00ffff, False, "main")
    # target above powLimit is rejected
    assert not native.check_proof_of_work(g, 0x1e00ffff, False, "main")
    # negative / zero targets rejected
    assert not native.check_proof_of_work(g, 0x01803456, False, "main")
    assert not native.check_proof_of_work(g, 0, False, "main")


# ------------------------------------------------------------------ merkle
def _py_merkle(leaves):
    if not leaves:
        return b"\x00" * 32, False
    level = list(leaves)
    mutated = False
    while len(level) > 1:
        for i in range(0, len(level) - 1, 2):
            if level[i] == level[i + 1]:
                mutated = True
        if len(level) % 2:
            level.append(level[-1])
        level = [sha256d(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
    return level[0], mutated


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 33, 100])
def test_merkle_root_matches_python(native, n):
    rng = random.Random(n)
    leaves = [rng.randbytes(32) for _ in range(n)]
    root, mut = native.merkle_root(leaves)
    exp, emut = _py_merkle(leaves)
    assert root == exp and mut == emut
    for pos in range(min(n, 6)):
        br = native.merkle_branch(leaves, pos)
        assert native.merkle_root_from_branch(leaves[pos], br, pos) == root


def test_merkle_mutation_detected(native):
    rng = random.Random(5)
    leaves = [rng.randbytes(32) for _ in range(6)]
    root6, mut6 = native.merkle_root(leaves)
    assert not mut6
    # CVE-2012-2459: duplicating the last two leaves yields the same root, flagged as mutated
    root8, mut8 = native.merkle_root(leaves + leaves[4:6])
    assert root8 == root6 and mut8


# ------------------------------------------------------------------ secp256k1
def test_pubkey_create_matches_oracle(native):
    rng = random.Random(1)
    for _ in range(8):
        sec = rng.randbytes(32)
        if not native.ec_seckey_verify(sec):
            continue
        for comp in (True, False):
            assert native.ec_pubkey_create(sec, comp) == ref.pubkey_from_secret(sec, comp)


def test_sign_matches_oracle(native):
    rng = random.Random(2)
    for i in range(8):
        sec = rng.randbytes(32)
        msg = rng.randbytes(32)
        r, s, recid = ref.sign(sec, msg)
        assert native.ec_sign(sec, msg) == ref.der_encode(r, s)
        extra = (i + 1).to_bytes(4, "little") + b"\x00" * 28
        r2, s2, _ = ref.sign(sec, msg, extra)
        assert native.ec_sign(sec, msg, i + 1) == ref.der_encode(r2, s2)
        pub = ref.pubkey_from_secret(sec)
        assert native.ec_verify(pub, native.ec_sign(sec, msg), msg)
        assert ref.verify(pub, r, s, msg)


def test_rfc6979_nonce(native):
    rng = random.Random(3)
    for c in range(3):
        k, m = rng.randbytes(32), rng.randbytes(32)
        assert native.ec_rfc6979_nonce(m, k, None, c) == ref.rfc6979_nonce(m, k, None, c)


def test_verify_rejects(native):
    rng = random.Random(4)
    sec, msg = rng.randbytes(32), rng.randbytes(32)
    pub = ref.pubkey_from_secret(sec)
    r, s, _ = ref.sign(sec, msg)
    good = ref.der_encode(r, s)
    assert native.ec_verify(pub, good, msg)
    # High-S is normalised by CPubKey::Verify (lax) -> still valid, but CheckLowS fails.
    high = ref.der_encode(r, ref.N - s)
    assert native.ec_verify(pub, high, msg)
    assert native.ec_check_low_s(good) and not native.ec_check_low_s(high)
    bad_msg = bytes([msg[0] ^ 1]) + msg[1:]
    assert not native.ec_verify(pub, good, bad_msg)
    assert not native.ec_verify(pub, b"", msg)
    assert not native.ec_verify(b"\x02" + b"\x00" * 32, good, msg)
    # uncompressed and hybrid encodings of the same key verify
    up = ref.pubkey_from_secret(sec, False)
    assert native.ec_verify(up, good, msg)
    hyb = bytes([6 + (up[64] & 1)]) + up[1:]
    assert native.ec_verify(hyb, good, msg)


def test_compact_recover(native):
    rng = random.Random(6)
    for comp in (True, False):
        sec, msg = rng.randbytes(32), rng.randbytes(32)
        sig = native.ec_sign_compact(sec, msg, comp)
        assert len(sig) == 65
        assert native.ec_recover_compact(msg, sig) == native.ec_pubkey_create(sec, comp)
        r = int.from_bytes(sig[1:33], "big")
        s = int.from_bytes(sig[33:], "big")
        rec = ref.recover(r, s, (sig[0] - 27) & 3, msg)
        assert ref.serialize_pubkey(rec, comp) == native.ec_pubkey_create(sec, comp)


# ------------------------------------------------------------------ key_tests (reference src/test/key_tests.cpp)
SECRET1 = "5HxWvvfubhXpYYpS3tJkw6fq9jE9j18THftkZjHHfmFiWtmAbrj"
SECRET2 = "5KC4ejrDjv152FGwP386VD1i2NYc5KkfSMyv1nGy1VGDxGHqVY3"
SECRET1C = "Kwr371tjA9u2rFSMZjTNun2PXXP3WPZu2afRHTcta6KxEUdm1vEw"
SECRET2C = "L3Hq7a8FEQwJkW1M2GNKDW28546Vp5miewcCzSqUD9kCAXrJdS3g"
ADDR = {SECRET1: "CfijQPpGx8Y1wXCezKDVtiVSPrYs1TqKcS", SECRET2: "CWYreGRKEf45tmDJru2G9zG5fPSN7JN6T1",
        SECRET1C: "CeGCRrDwqS9rZLCKzGmys6FLUede24ZV4o", SECRET2C: "CTtcbLKQtFW3tR4x2ADdqrbiJVfZQD9cFm"}


def test_key_vectors(native):
    assert native.decode_secret("CKhavDqXogc5u6bEBFjnyxWoUWtQudxmNf", "main") is None
    for wif, addr in ADDR.items():
        sec, comp = native.decode_secret(wif, "main")
        assert comp == (wif[0] in "KL")
        pub = native.ec_pubkey_create(sec, comp)
        h160 = hashlib.new("sha256", pub).digest()
        kind, h = native.decode_destination(addr, "main")
        assert kind == "pubkey"
        assert native.encode_destination("pubkey", native.hash160(pub), "main", False) == addr
        assert native.encode_secret(sec, comp, "main") == wif
        del h160, h


def _hash256(s):
    return sha256d(s.encode())


def test_deterministic_signatures(native):
    # reference src/test/key_tests.cpp:162-196
    msg = _hash256("Very deterministic message")
    s1, c1 = native.decode_secret(SECRET1, "main")
    s2, _ = native.decode_secret(SECRET2, "main")
    assert native.ec_sign(s1, msg).hex() == (
        "304402205dbbddda71772d95ce91cd2d14b592cfbc1dd0aabd6a394b6c2d377bbe59d31d022014ddda21494a4e221f0824f0"
        "b8b924c43fa43c0ad57dccdaa11f81a6bd4582f6")
    assert native.ec_sign(s2, msg).hex() == (
        "3044022052d8a32079c11e79db95af63bb9600c5b04f21a9ca33dc129c2bfa8ac9dc1cd5022061d8ae5e0f6c1a16bde3719c"
        "64c2fd70e404b6428ab9a69566962e8771b5944d")
    assert native.ec_sign_compact(s1, msg, False).hex() == (
        "1c5dbbddda71772d95ce91cd2d14b592cfbc1dd0aabd6a394b6c2d377bbe59d31d14ddda21494a4e221f0824f0b8b924c43f"
        "a43c0ad57dccdaa11f81a6bd4582f6")
    assert native.ec_sign_compact(s1, msg, True).hex() == (
        "205dbbddda71772d95ce91cd2d14b592cfbc1dd0aabd6a394b6c2d377bbe59d31d14ddda21494a4e221f0824f0b8b924c43f"
        "a43c0ad57dccdaa11f81a6bd4582f6")


def test_sign_verify_matrix(native):
    # reference src/test/key_tests.cpp:104-160
    keys = [native.decode_secret(w, "main") for w in (SECRET1, SECRET2, SECRET1C, SECRET2C)]
    pubs = [native.ec_pubkey_create(s, c) for s, c in keys]
    for n in range(4):
        msg = _hash256(f"Very secret message {n}: 11")
        sigs = [native.ec_sign(s, msg) for s, _ in keys]
        for i, pub in enumerate(pubs):
            for j, sig in enumerate(sigs):
                assert native.ec_verify(pub, sig, msg) == (i % 2 == j % 2)
        for (s, c), pub in zip(keys, pubs):
            assert native.ec_recover_compact(msg, native.ec_sign_compact(s, msg, c)) == pub


# ------------------------------------------------------------------ encodings
def test_base58_encode_decode_vectors(native):
    # reference src/test/base58_tests.cpp (base58_EncodeBase58, base58_DecodeBase58,
    # base58_keys_valid_parse/gen, base58_keys_invalid) over its own JSON vectors
    for hexstr, b58 in load_ref_json("base58_encode_decode.json"):
        assert native.base58_encode(bytes.fromhex(hexstr)) == b58
        assert native.base58_decode(b58) == bytes.fromhex(hexstr)
    assert native.base58_decode("invalid") is None
    assert native.base58_decode(" \t\n\v\f\r skip \r\f\v\n\t a") is None
    assert native.base58_decode(" \t\n\v\f\r 2g \r\f\v\n\t ") == b"a"


def test_base58_keys_valid(native):
    for b58, payload, meta in load_ref_json("base58_keys_valid.json"):
        chain = "test" if meta["isTestnet"] else "main"
        if meta["isPrivkey"]:
            r = native.decode_secret(b58, chain)
            assert r is not None, b58
            assert r[0].hex() == payload.lower() and r[1] == meta["isCompressed"]
            assert native.encode_secret(r[0], r[1], chain) == b58
        else:
            r = native.decode_destination(b58, chain)
            if meta["addrType"] == "none":
                continue
            assert r is not None, b58
            assert r[0] == meta["addrType"] and r[1].hex() == payload.lower()
            assert native.encode_destination(r[0], r[1], chain, False) == b58


def test_base58_keys_invalid(native):
    for (b58,) in load_ref_json("base58_keys_invalid.json"):
        for chain in ("main", "test"):
            assert native.decode_destination(b58, chain) is None
            assert native.decode_secret(b58, chain) is None


def test_cashaddr_vectors(native):
    # reference src/test/cashaddr_tests.cpp:40-72
    for s in ["prefix:x64nx6hz", "PREFIX:X64NX6HZ", "p:gpf8m4h7", "bitcoincash:qpzry9x8gf2tvdw0s3jn54khce6mua7lcw20ayyn",
              "bchtest:testnetaddress4d6njnut", "bchreg:555555555555555555555555555555555555555555555udxmlmrz"]:
        prefix, payload = native.cashaddr_decode(s, "")
        assert prefix == s.split(":")[0].lower()
        assert native.cashaddr_encode(prefix, payload) == s.lower()
    for s in ["prefix:x32nx6hz", "prEfix:x64nx6hz", "prefix:x64nx6Hz", "pref1x:6m8cxv73", "prefix:", ":u9wsx07j",
              "bchreg:555555555555555555x55555555555555555555555555udxmlmrz",
              "bchreg:555555555555555555555555555555551555555555555udxmlmrz", "pre:fix:x32nx6hz", "prefixx64nx6hz"]:
        assert native.cashaddr_decode(s, "")[0] == ""


def test_cashaddr_addresses(native):
    # reference src/test/cashaddrenc_tests.cpp:268-285
    h = bytes([0, 17, 128, 5, 246, 174, 201, 130, 217, 236, 131, 136, 199, 148, 26, 202, 163, 58, 140, 221])
    pk = "bitcoincashplus:qqqprqq976hvnqkeajpc33u5rt92xw5vm5ylgfku0f"
    sc = "bitcoincashplus:pqqprqq976hvnqkeajpc33u5rt92xw5vm5n64x3l55"
    assert native.encode_destination("pubkey", h, "main", True) == pk
    assert native.encode_destination("script", h, "main", True) == sc
    assert native.decode_destination(pk, "main") == ("pubkey", h)
    assert native.decode_destination(sc, "main") == ("script", h)
    # prefix is optional on decode for the active network, upper case accepted
    assert native.decode_destination(pk.split(":")[1], "main") == ("pubkey", h)
    assert native.decode_destination(pk.upper(), "main") == ("pubkey", h)
    # wrong network prefix
    assert native.decode_destination(pk, "test") is None


def test_bip32_vector1(native):
    # BIP32 test vector 1 (public spec); xprv/xpub use the main-net version bytes.
    seed = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    xprv, xpub = native.bip32_master(seed, "main")
    assert xpub == "xpub661MyMwAqRbcFtXgS5sYJABqqG9YLmC4Q1Rdap9gSE8NqtwybGhePY2gZ29ESFjqJoCu1Rupje8YtGqsefD265TMg7usUDFdp6W1EGMcet8"
    assert xprv == "xprv9s21ZrQH143K3QTDL4LXw2F7HEK3wJUD2nW2nRk4stbPy6cq3jPPqjiChkVvvNKmPGJxWUtg6LnF5kejMRNNU3TGtRBeJgk33yuGBxrMPHi"
    xprv1, xpub1 = native.bip32_derive(xprv, 0x80000000, "main")
    assert xpub1 == "xpub68Gmy5EdvgibQVfPdqkBBCHxA5htiqg55crXYuXoQRKfDBFA1WEjWgP6LHhwBZeNK1VTsfTFUHCdrfp1bgwQ9xv5ski8PX9rL2dZXvgGDnw"
    xprv2, xpub2 = native.bip32_derive(xprv1, 1, "main")
    assert xpub2 == "xpub6ASuArnXKPbfEwhqN6e3mwBcDTgzisQN1wXN9BJcM47sSikHjJf3UFHKkNAWbWMiGj7Wf5uMash7SyYq527Hqck2AxYysAA7xmALppuCkwQ"
    # public derivation of a non-hardened child matches the private path
    assert native.bip32_derive_pub(xpub1, 1, "main") == xpub2


# reference src/test/bip32_tests.cpp test1 / test2: (xpub, xprv, index of the next derivation)
BIP32_VECTORS = [
    ("000102030405060708090a0b0c0d0e0f", [
        ("xpub661MyMwAqRbcFtXgS5sYJABqqG9YLmC4Q1Rdap9gSE8NqtwybGhePY2gZ29ESFjqJoCu1Rupje8YtGqsefD265TMg7usUDFdp6W1EGMcet8",
         "xprv9s21ZrQH143K3QTDL4LXw2F7HEK3wJUD2nW2nRk4stbPy6cq3jPPqjiChkVvvNKmPGJxWUtg6LnF5kejMRNNU3TGtRBeJgk33yuGBxrMPHi",
         0x80000000),
        ("xpub68Gmy5EdvgibQVfPdqkBBCHxA5htiqg55crXYuXoQRKfDBFA1WEjWgP6LHhwBZeNK1VTsfTFUHCdrfp1bgwQ9xv5ski8PX9rL2dZXvgGDnw",
         "xprv9uHRZZhk6KAJC1avXpDAp4MDc3sQKNxDiPvvkX8Br5ngLNv1TxvUxt4cV1rGL5hj6KCesnDYUhd7oWgT11eZG7XnxHrnYeSvkzY7d2bhkJ7",
         1),
        ("xpub6ASuArnXKPbfEwhqN6e3mwBcDTgzisQN1wXN9BJcM47sSikHjJf3UFHKkNAWbWMiGj7Wf5uMash7SyYq527Hqck2AxYysAA7xmALppuCkwQ",
         "xprv9wTYmMFdV23N2TdNG573QoEsfRrWKQgWeibmLntzniatZvR9BmLnvSxqu53Kw1UmYPxLgboyZQaXwTCg8MSY3H2EU4pWcQDnRnrVA1xe8fs",
         0x80000002),
        ("xpub6D4BDPcP2GT577Vvch3R8wDkScZWzQzMMUm3PWbmWvVJrZwQY4VUNgqFJPMM3No2dFDFGTsxxpG5uJh7n7epu4trkrX7x7DogT5Uv6fcLW5",
         "xprv9z4pot5VBttmtdRTWfWQmoH1taj2axGVzFqSb8C9xaxKymcFzXBDptWmT7FwuEzG3ryjH4ktypQSAewRiNMjANTtpgP4mLTj34bhnZX7UiM",
         2),
        ("xpub6FHa3pjLCk84BayeJxFW2SP4XRrFd1JYnxeLeU8EqN3vDfZmbqBqaGJAyiLjTAwm6ZLRQUMv1ZACTj37sR62cfN7fe5JnJ7dh8zL4fiyLHV",
         "xprvA2JDeKCSNNZky6uBCviVfJSKyQ1mDYahRjijr5idH2WwLsEd4Hsb2Tyh8RfQMuPh7f7RtyzTtdrbdqqsunu5Mm3wDvUAKRHSC34sJ7in334",
         1000000000),
        ("xpub6H1LXWLaKsWFhvm6RVpEL9P4KfRZSW7abD2ttkWP3SSQvnyA8FSVqNTEcYFgJS2UaFcxupHiYkro49S8yGasTvXEYBVPamhGW6cFJodrTHy",
         "xprvA41z7zogVVwxVSgdKUHDy1SKmdb533PjDz7J6N6mV6uS3ze1ai8FHa8kmHScGpWmj4WggLyQjgPie1rFSruoUihUZREPSL39UNdE3BBDu76",
         None),
    ]),
    ("fffcf9f6f3f0edeae7e4e1dedbd8d5d2cfccc9c6c3c0bdbab7b4b1aeaba8a5a29f9c999693908d8a8784817e7b7875726f6c696663605d5a5754514e4b484542", [
        ("xpub661MyMwAqRbcFW31YEwpkMuc5THy2PSt5bDMsktWQcFF8syAmRUapSCGu8ED9W6oDMSgv6Zz8idoc4a6mr8BDzTJY47LJhkJ8UB7WEGuduB",
         "xprv9s21ZrQH143K31xYSDQpPDxsXRTUcvj2iNHm5NUtrGiGG5e2DtALGdso3pGz6ssrdK4PFmM8NSpSBHNqPqm55Qn3LqFtT2emdEXVYsCzC2U",
         0),
        ("xpub69H7F5d8KSRgmmdJg2KhpAK8SR3DjMwAdkxj3ZuxV27CprR9LgpeyGmXUbC6wb7ERfvrnKZjXoUmmDznezpbZb7ap6r1D3tgFxHmwMkQTPH",
         "xprv9vHkqa6EV4sPZHYqZznhT2NPtPCjKuDKGY38FBWLvgaDx45zo9WQRUT3dKYnjwih2yJD9mkrocEZXo1ex8G81dwSM1fwqWpWkeS3v86pgKt",
         0xFFFFFFFF),
        ("xpub6ASAVgeehLbnwdqV6UKMHVzgqAG8Gr6riv3Fxxpj8ksbH9ebxaEyBLZ85ySDhKiLDBrQSARLq1uNRts8RuJiHjaDMBU4Zn9h8LZNnBC5y4a",
         "xprv9wSp6B7kry3Vj9m1zSnLvN3xH8RdsPP1Mh7fAaR7aRLcQMKTR2vidYEeEg2mUCTAwCd6vnxVrcjfy2kRgVsFawNzmjuHc2YmYRmagcEPdU9",
         1),
        ("xpub6DF8uhdarytz3FWdA8TvFSvvAh8dP3283MY7p2V4SeE2wyWmG5mg5EwVvmdMVCQcoNJxGoWaU9DCWh89LojfZ537wTfunKau47EL2dhHKon",
         "xprv9zFnWC6h2cLgpmSA46vutJzBcfJ8yaJGg8cX1e5StJh45BBciYTRXSd25UEPVuesF9yog62tGAQtHjXajPPdbRCHuWS6T8XA2ECKADdw4Ef",
         0xFFFFFFFE),
        ("xpub6ERApfZwUNrhLCkDtcHTcxd75RbzS1ed54G1LkBUHQVHQKqhMkhgbmJbZRkrgZw4koxb5JaHWkY4ALHY2grBGRjaDMzQLcgJvLJuZZvRcEL",
         "xprvA1RpRA33e1JQ7ifknakTFpgNXPmW2YvmhqLQYMmrj4xJXXWYpDPS3xz7iAxn8L39njGVyuoseXzU6rcxFLJ8HFsTjSyQbLYnMpCqE2VbFWc",
         2),
        ("xpub6FnCn6nSzZAw5Tw7cgR9bi15UV96gLZhjDstkXXxvCLsUXBGXPdSnLFbdpq8p9HmGsApME5hQTZ3emM2rnY5agb9rXpVGyy3bdW6EEgAtqt",
         "xprvA2nrNbFZABcdryreWet9Ea4LvTJcGsqrMzxHx98MMrotbir7yrKCEXw7nadnHM8Dq38EGfSh6dqA9QWTyefMLEcBYJUuekgW4BYPJcr9E7j",
         None),
    ]),
]


def test_bip32_reference_vectors(native):
    """reference src/test/bip32_tests.cpp (bip32_test1, bip32_test2): the master key from each seed
    and every derivation step, private and (for non-hardened steps) public."""
    for seed, steps in BIP32_VECTORS:
        xprv, xpub = native.bip32_master(bytes.fromhex(seed), "main")
        for want_pub, want_prv, nxt in steps:
            assert (xpub, xprv) == (want_pub, want_prv)
            if nxt is None:
                break
            nprv, npub = native.bip32_derive(xprv, nxt, "main")
            if not nxt & 0x80000000:
                assert native.bip32_derive_pub(xpub, nxt, "main") == npub
            xprv, xpub = nprv, npub


def test_message_hash(native):
    magic = b"Bitcoin Signed Message:\n"
    msg = b"hello"
    exp = sha256d(bytes([len(magic)]) + magic + bytes([len(msg)]) + msg)
    assert native.message_hash("hello") == exp


def test_lockorder_detector(native):
    # first order a->b is recorded silently; the reverse b->a is reported (reference sync.cpp
    # potential_deadlock_detected)
    first, total = native.lockorder_probe()
    assert (first, total) == (0, 1)
