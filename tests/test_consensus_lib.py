"""libbcpconsensus C API (reference src/script/bitcoinconsensus.{h,cpp}) via ctypes.

Vectors are built with bcp-tx from the reference's txcreatesignv1 inputs (privkey 1,
P2PKH 76a91491b2...), but with sign= issued after the outputs are added. (The reference
vector itself signs before `outaddr=` runs, so its signature does not commit to the final
outputs and is invalid by construction; bcp-tx reproduces that byte-for-byte.)"""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lib", "libbcpconsensus.so")
if not os.path.exists(LIB):
    subprocess.check_call(["make", "-C", ROOT, "-j8", "conslib"])

SPK = bytes.fromhex("76a91491b24bf9f5288532960ac687abb035127b1d28a588ac")
TXID = "4d49a71ec9da436f71ec4ee231d04f292a29cd316f598bb7068feccabdc59485"


def _build(sighash, amount=None):
    prev = '[{"txid":"%s","vout":0,"scriptPubKey":"%s"%s}]' % (TXID, SPK.hex(), "" if amount is None else ',"amount":%s' % amount)
    out = subprocess.run([os.path.join(ROOT, "bin", "bcp-tx"), "-create", "nversion=1", f"in={TXID}:0",
                          "outaddr=0.001:CGWgb1vrYoMVW4Eqnfbmr1UYSotuHXnvKA",
                          'set=privatekeys:["5HpHagT65TZzG1PH3CSu63k8DbpvD8s5ip4nEB3kEsreAnchuDf"]',
                          "set=prevtxs:" + prev, "sign=" + sighash], capture_output=True, text=True, check=True)
    return bytes.fromhex(out.stdout.strip())


TX = _build("ALL")
TXF = _build("ALL|FORKID", "0.002")
P2SH, FORKID = 1 << 0, 1 << 16


@pytest.fixture(scope="module")
def lib():
    l = ctypes.CDLL(LIB)
    l.bitcoinconsensus_verify_script.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_char_p, ctypes.c_uint,
                                                 ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(ctypes.c_int)]
    l.bitcoinconsensus_verify_script_with_amount.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_int64,
                                                             ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint,
                                                             ctypes.c_uint, ctypes.POINTER(ctypes.c_int)]
    return l


def call(lib, spk, tx, n=0, flags=P2SH, amount=None):
    err = ctypes.c_int(-1)
    if amount is None:
        r = lib.bitcoinconsensus_verify_script(spk, len(spk), tx, len(tx), n, flags, ctypes.byref(err))
    else:
        r = lib.bitcoinconsensus_verify_script_with_amount(spk, len(spk), amount, tx, len(tx), n, flags,
                                                          ctypes.byref(err))
    return r, err.value


def test_version(lib):
    assert lib.bitcoinconsensus_version() == 1


def test_valid_legacy_spend(lib):
    assert call(lib, SPK, TX) == (1, 0)
    assert call(lib, SPK, TX, amount=100000) == (1, 0)


def test_invalid(lib):
    bad_spk = SPK[:5] + bytes([SPK[5] ^ 1]) + SPK[6:]
    assert call(lib, bad_spk, TX)[0] == 0
    # FORKID enforced: a legacy signature no longer verifies
    assert call(lib, SPK, TX, flags=P2SH | FORKID, amount=100000)[0] == 0


def test_forkid_spend_commits_to_amount(lib):
    assert call(lib, SPK, TXF, flags=P2SH | FORKID, amount=200000) == (1, 0)
    assert call(lib, SPK, TXF, flags=P2SH | FORKID, amount=200001)[0] == 0


def test_errors(lib):
    assert call(lib, SPK, TX, n=1) == (0, 1)                       # ERR_TX_INDEX
    assert call(lib, SPK, TX + b"\x00") == (0, 2)                  # ERR_TX_SIZE_MISMATCH
    assert call(lib, SPK, TX[:20]) == (0, 3)                       # ERR_TX_DESERIALIZE
    assert call(lib, SPK, TX, flags=FORKID) == (0, 4)              # ERR_AMOUNT_REQUIRED
    assert call(lib, SPK, TX, flags=1 << 1) == (0, 5)              # ERR_INVALID_FLAGS
